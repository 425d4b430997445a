// packed.hip -- Golay(24,12) and Hamming(8,4) over packed storage (SURVEY
// §8f rank 3).
//
// The reference's layout spends 4 B on a 24-bit codeword (int32) and 1 B on a
// 4-bit value (uint8 triplets), so its decode moves 8 B per codeword.  This is
// an additional, native layout -- not a replacement of the reference API:
//   * values:    INT4 nibbles two per byte, value j in byte j/2 (low nibble
//                first), so codeword k's 12 data bits are bits 12k..12k+11 of
//                the little-endian nibble stream;
//   * codewords: 3 little-endian bytes each (bits 24k..24k+23 of the stream),
//                same bit layout as the reference's data12 | parity12 << 12;
//   * decode flags: one bit per codeword (1 = uncorrectable, data kept), eight
//                codewords per byte.
// Decode moves 3 + 1.5 + 0.125 = 4.625 B per codeword, encode 1.5 + 3 = 4.5 B.
// Hamming(8,4) keeps its byte codewords (already 8 bits) but packs the values
// (nibbles) and the decode's ErrorType (2 bits per value, value j at bits
// 2(j%4) of byte j/4): encode 0.5 + 1 = 1.5 B/value, decode 1 + 0.5 + 0.25 =
// 1.75 B/value (reference layout: 2 and 3).
//
// gfx950 design: a lane owns groups of 8 codewords = 12 B of nibbles + 24 B of
// codewords (word aligned), kPkGroups groups per lane per tile.  Every
// wave-instruction covers one contiguous span: nibbles move as 12 B per lane;
// encode stores codewords as a 16 B + 8 B pair per lane regrouped through LDS
// (with a plain 24 B lane stride packed encode ran at 3.4 TB/s).
// Parity / correction tables in LDS as in golay.hip; all HBM accesses
// non-temporal.
#include "kvecc_internal.h"

namespace kvecc {

constexpr int kPkGroups = 2;
constexpr int kPkBlock = 512;
constexpr int kPkTile = kPkBlock * kPkGroups * 8;  // codewords per workgroup tile
constexpr int kPkWaveCw = kWave * kPkGroups * 8;

// 12 data words of a group <-> 3 nibble words (96 bits)
__device__ __forceinline__ void nib_unpack8(const uint32_t n[3], uint32_t d[8]) {
  d[0] = n[0] & 0xFFFu;
  d[1] = (n[0] >> 12) & 0xFFFu;
  d[2] = (n[0] >> 24) | (n[1] & 0xFu) << 8;
  d[3] = (n[1] >> 4) & 0xFFFu;
  d[4] = (n[1] >> 16) & 0xFFFu;
  d[5] = (n[1] >> 28) | (n[2] & 0xFFu) << 4;
  d[6] = (n[2] >> 8) & 0xFFFu;
  d[7] = n[2] >> 20;
}
__device__ __forceinline__ void nib_pack8(const uint32_t d[8], uint32_t n[3]) {
  n[0] = d[0] | d[1] << 12 | d[2] << 24;
  n[1] = d[2] >> 8 | d[3] << 4 | d[4] << 16 | d[5] << 28;
  n[2] = d[5] >> 4 | d[6] << 8 | d[7] << 20;
}
// 8 24-bit codewords <-> 6 words (192 bits)
__device__ __forceinline__ void cw_unpack8(const uint32_t w[6], uint32_t c[8]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t a = w[3 * h], b = w[3 * h + 1], e = w[3 * h + 2];
    c[4 * h + 0] = a & 0xFFFFFFu;
    c[4 * h + 1] = (a >> 24) | (b & 0xFFFFu) << 8;
    c[4 * h + 2] = (b >> 16) | (e & 0xFFu) << 16;
    c[4 * h + 3] = e >> 8;
  }
}
__device__ __forceinline__ void cw_pack8(const uint32_t c[8], uint32_t w[6]) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t *x = c + 4 * h;
    w[3 * h] = x[0] | x[1] << 24;
    w[3 * h + 1] = x[1] >> 8 | x[2] << 16;
    w[3 * h + 2] = x[2] >> 16 | x[3] << 8;
  }
}

__device__ __forceinline__ void load_tables_pk(uint16_t *lds, const uint16_t *par,
                                               const uint16_t *cor, bool need_cor) {
  const u32x4 *p = reinterpret_cast<const u32x4 *>(par);
  u32x4 *l = reinterpret_cast<u32x4 *>(lds);
  for (int i = threadIdx.x; i < 512; i += kPkBlock) l[i] = p[i];
  if (need_cor) {
    const u32x4 *c = reinterpret_cast<const u32x4 *>(cor);
    for (int i = threadIdx.x; i < 512; i += kPkBlock) l[512 + i] = c[i];
  }
  __syncthreads();
}

// A wave's 64 groups of codewords are 1536 contiguous bytes: in HBM they move as
// one 16-byte and one 8-byte access per lane (1024 + 512 B, each contiguous
// across the wave) and are regrouped to 24 bytes per lane through LDS.
constexpr int kWaveCwBytes = kWave * 24;
typedef uint32_t u32x3v __attribute__((ext_vector_type(3)));

__global__ __launch_bounds__(kPkBlock) void golay_encode_packed_kernel(
    const uint32_t *__restrict__ nib, uint32_t *__restrict__ cw, int64_t ntiles,
    const uint16_t *__restrict__ par) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[4096];
  __shared__ __attribute__((aligned(16))) uint8_t stage[kPkBlock / kWave][kPkGroups][kWaveCwBytes];
  load_tables_pk(lds, par, nullptr, false);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t G0 = (t * kPkTile + wave * kPkWaveCw) / 8;  // first group of this wave
    u32x3v n[kPkGroups];
#pragma unroll
    for (int g = 0; g < kPkGroups; ++g)
      n[g] = ld_stream(reinterpret_cast<const u32x3v *>(nib + (G0 + g * kWave + lane) * 3));
#pragma unroll
    for (int g = 0; g < kPkGroups; ++g) {
      const uint32_t nn[3] = {n[g].x, n[g].y, n[g].z};
      uint32_t d[8], c[8], w[6];
      nib_unpack8(nn, d);
#pragma unroll
      for (int k = 0; k < 8; ++k) c[k] = d[k] | (uint32_t)lds[d[k]] << 12;
      cw_pack8(c, w);
      u32x2 *dst = reinterpret_cast<u32x2 *>(&stage[wave][g][24 * lane]);
      dst[0] = u32x2{w[0], w[1]};
      dst[1] = u32x2{w[2], w[3]};
      dst[2] = u32x2{w[4], w[5]};
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < kPkGroups; ++g) {
      uint8_t *out = reinterpret_cast<uint8_t *>(cw) + (G0 + g * kWave) * 24;
      st_stream(reinterpret_cast<u32x4 *>(out) + lane,
                *reinterpret_cast<const u32x4 *>(&stage[wave][g][16 * lane]));
      st_stream(reinterpret_cast<u32x2 *>(out + 1024) + lane,
                *reinterpret_cast<const u32x2 *>(&stage[wave][g][1024 + 8 * lane]));
    }
    __syncthreads();
  }
}

// decode reads its 24 B per lane directly as three 8-byte loads (the three
// instructions of a wave together cover the wave's 1536 contiguous bytes);
// regrouping through LDS as in encode measured slower here (48 vs 44 us)
template <bool WITH_FLAGS, bool WITH_STATS>
__global__ __launch_bounds__(kPkBlock) void golay_decode_packed_kernel(
    const uint32_t *__restrict__ cw, uint32_t *__restrict__ nib, uint8_t *__restrict__ flags,
    int64_t ntiles, const uint16_t *__restrict__ par, const uint16_t *__restrict__ cor,
    uint64_t *__restrict__ stats) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[8192];
  load_tables_pk(lds, par, cor, true);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  uint32_t bits = 0, unc = 0;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t G0 = (t * kPkTile + wave * kPkWaveCw) / 8;
    u32x2 p[kPkGroups][3];
#pragma unroll
    for (int g = 0; g < kPkGroups; ++g) {
      const u32x2 *src = reinterpret_cast<const u32x2 *>(cw + (G0 + g * kWave + lane) * 6);
#pragma unroll
      for (int k = 0; k < 3; ++k) p[g][k] = ld_stream(src + k);
    }
#pragma unroll
    for (int g = 0; g < kPkGroups; ++g) {
      const uint32_t w[6] = {p[g][0].x, p[g][0].y, p[g][1].x, p[g][1].y, p[g][2].x, p[g][2].y};
      uint32_t c[8], d[8], n[3], fl = 0;
      cw_unpack8(w, c);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint32_t cnt;
        d[k] = golay_decode1(c[k], lds, lds + 4096, cnt);
        bits += cnt & 3u;
        unc += cnt >> 2;
        fl |= (cnt >> 2) << k;
      }
      nib_pack8(d, n);
      st_stream(reinterpret_cast<u32x3v *>(nib + (G0 + g * kWave + lane) * 3), u32x3v{n[0], n[1], n[2]});
      if (WITH_FLAGS) st_stream(flags + G0 + g * kWave + lane, (uint8_t)fl);
    }
    wave_lds_sync();
  }
  if (WITH_STATS) flush_stats2<kPkBlock>(stats, bits, unc);
}

// Staged variant: each wave loads its 3072 contiguous codeword bytes (two
// groups of 8 codewords per lane) as three 16-byte loads per lane into a
// wave-private LDS region -- no workgroup barrier -- with the next tile's loads
// already in registers, and reads its 24-byte groups back as 8-byte LDS reads
// (lane stride 6 dwords: conflict-free).  43.6 vs 44.9 us for the direct
// 8-byte-load kernel above (tools/exp/run_packed.py); taken for 16-B aligned
// codewords past the wave-tile kernel's 2 GiB range.
// workgroups per CU of the decode grid (a cap: smaller grids loop over tiles,
// staging the 16 KiB of tables once per workgroup instead of once per tile)
constexpr int kPkDecPerCu = 32;
constexpr int kPkWaveBytes = kPkWaveCw * 3;  // 3072
template <bool WITH_FLAGS, bool WITH_STATS>
__global__ __launch_bounds__(kPkBlock) void golay_decode_packed_staged_kernel(
    const uint32_t *__restrict__ cw, uint32_t *__restrict__ nib, uint8_t *__restrict__ flags,
    int64_t ntiles, const uint16_t *__restrict__ par, const uint16_t *__restrict__ cor,
    uint64_t *__restrict__ stats) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[8192];
  __shared__ __attribute__((aligned(16))) uint8_t stage[kPkBlock / kWave][kPkWaveBytes];
  load_tables_pk(lds, par, cor, true);
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  uint8_t *mine = stage[wave];
  uint32_t bits = 0, unc = 0;
  constexpr int kV = kPkWaveBytes / 16 / kWave;  // 3 vectors per lane
  auto src_of = [&](int64_t t) {
    return reinterpret_cast<const u32x4 *>(reinterpret_cast<const uint8_t *>(cw) +
                                           (t * kPkTile + wave * kPkWaveCw) * 3);
  };
  u32x4 nxt[kV];
  int64_t t = blockIdx.x;
  if (t < ntiles) {
#pragma unroll
    for (int k = 0; k < kV; ++k) nxt[k] = ld_stream(src_of(t) + lane + k * kWave);
  }
  for (; t < ntiles; t += gridDim.x) {
#pragma unroll
    for (int k = 0; k < kV; ++k) reinterpret_cast<u32x4 *>(mine)[lane + k * kWave] = nxt[k];
    // lanes read each other's bytes through other vector types: keep the
    // compiler from moving LDS accesses across the phase boundaries
    wave_lds_sync();
    if (t + gridDim.x < ntiles) {
#pragma unroll
      for (int k = 0; k < kV; ++k) nxt[k] = ld_stream(src_of(t + gridDim.x) + lane + k * kWave);
    }
    const int64_t G0 = (t * kPkTile + wave * kPkWaveCw) / 8;
#pragma unroll
    for (int g = 0; g < kPkGroups; ++g) {
      const u32x2 *p = reinterpret_cast<const u32x2 *>(mine + (g * kWave + lane) * 24);
      const u32x2 a = p[0], b = p[1], c2 = p[2];
      const uint32_t w[6] = {a.x, a.y, b.x, b.y, c2.x, c2.y};
      uint32_t c[8], d[8], n[3], fl = 0;
      cw_unpack8(w, c);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        uint32_t cnt;
        d[k] = golay_decode1(c[k], lds, lds + 4096, cnt);
        bits += cnt & 3u;
        unc += cnt >> 2;
        fl |= (cnt >> 2) << k;
      }
      nib_pack8(d, n);
      st_stream(reinterpret_cast<u32x3v *>(nib + (G0 + g * kWave + lane) * 3), u32x3v{n[0], n[1], n[2]});
      if (WITH_FLAGS) st_stream(flags + G0 + g * kWave + lane, (uint8_t)fl);
    }
    wave_lds_sync();
  }
  if (WITH_STATS) flush_stats2<kPkBlock>(stats, bits, unc);
}

// Wave-tile decode (the default): a wave owns tiles of 1024 codewords (3072
// codeword bytes in, 1536 nibble bytes + 128 flag bytes out), scheduled as the
// fused reads are (TileSchedule: a static share, then per-launch counters), so
// the grid is persistent -- 3 workgroups per CU, each staging its 24 KiB of
// tables once -- and no wave waits on another.  The tile's bytes come in as
// three 16-byte buffer loads per lane (each wave-instruction 1 KiB
// contiguous), the next tile's already in flight, through a wave-private LDS
// stage; each lane then decodes two groups of 8 codewords.  Per codeword: one
// lookup of parity(lo) << 2 (a byte offset), one of the syndrome's entry
// (error data | bits << 24 | uncorrectable << 31), data = (c ^ e) & 0xFFF in one
// v_bitop3, the statistics as a 32-bit sum of entries (bits 24-30: corrected
// bits of <= 8 codewords) and the flag bits shifted in with v_alignbit.
// workgroups per CU of the persistent grid, and the dynamic tail's static
// share: 2 per CU and 50 % measured 34.8-35.0 us against 35.0-35.3 at 75 %; 3
// per CU (any share), 256- and 384-thread workgroups, LDS-DMA staging and
// conflict-free table addresses were all no faster (profiles/r04/packed_dec_ab_*.log)
constexpr int kPk2PerCu = 2;
constexpr uint32_t kPk2StaticPct = 50;
constexpr int kPk2Block = 512;
constexpr int kPk2Waves = kPk2Block / kWave;
// groups of 8 codewords per lane per wave tile (2: 1024 codewords, 3 KiB);
// 4 and 6 measured 41.0 and 52.4 us against 39.2 (profiles/r03/packed/pk_ab7.log)
constexpr int kPk2Groups = 2;
constexpr int kPk2TileCw = kWave * 8 * kPk2Groups;  // codewords per wave tile
constexpr int kPk2TileBytes = kPk2TileCw * 3;       // 3 KiB per 2 groups
constexpr int kPk2Vec = kPk2TileBytes / 16 / kWave;  // 16-byte loads per lane
// The uncorrectable flags (one byte per group of 8 codewords, one byte store
// per lane per group) staged in LDS and stored 16 bytes per lane instead
// measured no faster (38.4 vs 38.1 us, profiles/r03/packed/pk_flags16_ab.log).
struct PkDecArgs {
  const uint8_t *cw;
  uint32_t *nib;
  uint8_t *flags;
  uint32_t units;  // wave tiles
  const uint8_t *tab;  // golay_pk_table_dev()
  uint64_t *stats;
  uint32_t *dyn;
};

template <bool WITH_FLAGS, bool WITH_STATS>
__global__ __launch_bounds__(kPk2Block) void golay_decode_packed_wave_kernel(PkDecArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t tab[24576];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kPk2Waves][kPk2TileBytes];
  for (int i = threadIdx.x; i < 24576 / 16; i += kPk2Block)
    reinterpret_cast<u32x4 *>(tab)[i] = reinterpret_cast<const u32x4 *>(a.tab)[i];
  __syncthreads();
  const uint32_t wave = uni((uint32_t)threadIdx.x / kWave), lane = threadIdx.x % kWave;
  const uint32_t gw = blockIdx.x * kPk2Waves + wave, nwaves = gridDim.x * kPk2Waves;
  if (gw >= a.units) return;  // no workgroup barrier below
  uint8_t *stage = stage_all[wave];
  TileSchedule sched;
  sched.init(a.units, a.dyn, gw, nwaves, lane, kPk2StaticPct);
  // whole codeword buffer (< 2 GiB, checked on the host); nt loads
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t *>(a.cw), 0, (int)(a.units * (uint32_t)kPk2TileBytes), 0x00020000);
  uint32_t t = gw;
  u32x4 nxt[kPk2Vec];
  auto issue = [&](uint32_t tt) {
#pragma unroll
    for (int k = 0; k < kPk2Vec; ++k)
      nxt[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                             rs, tt * (uint32_t)kPk2TileBytes + 16u * (lane + kWave * k), 0, 2));
  };
  issue(t);
  uint32_t bits = 0, unc = 0;
  for (;;) {
#pragma unroll
    for (int k = 0; k < kPk2Vec; ++k) reinterpret_cast<u32x4 *>(stage)[lane + kWave * k] = nxt[k];
    wave_lds_sync();
    const uint32_t cur = t;
    t = sched.next(t, lane);
    const bool more = t < a.units;
    if (more) issue(t);
#pragma unroll
    for (int g = 0; g < kPk2Groups; ++g) {
      const u32x2 *p = reinterpret_cast<const u32x2 *>(stage + (g * kWave + lane) * 24);
      const u32x2 x0 = p[0], x1 = p[1], x2 = p[2];
      const uint32_t w[6] = {x0.x, x0.y, x1.x, x1.y, x2.x, x2.y};
      uint32_t c[8];  // bits 24-31 are a neighbour's: every use below masks them
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        c[4 * h] = w[3 * h];
        c[4 * h + 1] = __builtin_amdgcn_alignbyte(w[3 * h + 1], w[3 * h], 3);
        c[4 * h + 2] = __builtin_amdgcn_alignbyte(w[3 * h + 2], w[3 * h + 1], 2);
        c[4 * h + 3] = w[3 * h + 2] >> 8;
      }
      uint32_t d[8], esum = 0, fl = 0;
#pragma unroll
      for (int k = 7; k >= 0; --k) {  // descending: the flag of codeword k lands at bit k
        const uint32_t pv = *reinterpret_cast<const uint16_t *>(tab + ((c[k] << 1) & 0x1FFEu));
        const uint32_t off = __builtin_amdgcn_bitop3_b32(c[k] >> 10, pv, 0x3FFCu, 0x28);  // (S0 ^ S1) & S2
        const uint32_t e = *reinterpret_cast<const uint32_t *>(tab + 8192 + off);
        d[k] = __builtin_amdgcn_bitop3_b32(c[k], e, 0xFFFu, 0x28);
        esum += e;
        fl = __builtin_amdgcn_alignbit(fl, e, 31);  // fl << 1 | e >> 31
      }
      if (WITH_STATS) {
        bits += (esum >> 24) & 0x7Fu;  // <= 8 * 3; bit 31 collects the flags, dropped
        unc += __builtin_popcount(fl);
      }
      uint32_t n[3];
      nib_pack8(d, n);
      const uint32_t grp = cur * (kPk2TileCw / 8) + g * kWave + lane;  // group of 8 codewords
      st_stream(reinterpret_cast<u32x3v *>(a.nib + (size_t)grp * 3), u32x3v{n[0], n[1], n[2]});
      if (WITH_FLAGS) st_stream(a.flags + grp, (uint8_t)fl);
    }
    if (!more) break;
    wave_lds_sync();
  }
  if (WITH_STATS) {
    bits = wave_sum(bits);
    unc = wave_sum(unc);
    if (lane == 0) {
      uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
      if (bits) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)bits);
      if (unc) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)unc);
    }
  }
}

// ---- scalar tails (< one tile), byte accesses -----------------------------------

__device__ __forceinline__ uint32_t get_nib(const uint8_t *p, int64_t j) {
  return (p[j >> 1] >> (4 * (j & 1))) & 0xFu;
}
// encode: one thread per codeword (nibble bytes are only read)
__global__ __launch_bounds__(kBlock) void golay_encode_packed_tail_kernel(
    const uint8_t *__restrict__ nib, uint8_t *__restrict__ cw, int64_t begin, int64_t m,
    const uint16_t *__restrict__ par) {
  const int64_t k = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x;
  if (k >= m) return;
  const uint32_t d = get_nib(nib, 3 * k) | get_nib(nib, 3 * k + 1) << 4 | get_nib(nib, 3 * k + 2) << 8;
  const uint32_t c = d | (uint32_t)par[d] << 12;
  cw[3 * k] = (uint8_t)c;
  cw[3 * k + 1] = (uint8_t)(c >> 8);
  cw[3 * k + 2] = (uint8_t)(c >> 16);
}

// decode: one thread per group of 8 codewords (12 nibble bytes + 1 flag byte,
// never shared between groups because `begin` is a multiple of 8)
template <bool WITH_FLAGS, bool WITH_STATS>
__global__ __launch_bounds__(kBlock) void golay_decode_packed_tail_kernel(
    const uint8_t *__restrict__ cw, uint8_t *__restrict__ nib, uint8_t *__restrict__ flags,
    int64_t begin, int64_t m, const uint16_t *__restrict__ par, const uint16_t *__restrict__ cor,
    uint64_t *__restrict__ stats) {
  uint32_t bits = 0, unc = 0;
  for (int64_t g = begin / 8 + (int64_t)blockIdx.x * kBlock + threadIdx.x; g * 8 < m;
       g += (int64_t)gridDim.x * kBlock) {
    uint32_t fl = 0;
    for (int64_t k = g * 8; k < m && k < g * 8 + 8; ++k) {
      const uint32_t c = cw[3 * k] | (uint32_t)cw[3 * k + 1] << 8 | (uint32_t)cw[3 * k + 2] << 16;
      uint32_t cnt;
      const uint32_t d = golay_decode1(c, par, cor, cnt);
      bits += cnt & 3u;
      unc += cnt >> 2;
      fl |= (cnt >> 2) << (k - g * 8);
      for (int e = 0; e < 3; ++e) {
        const int64_t j = 3 * k + e;
        const uint32_t v = d >> (4 * e) & 0xFu;
        if ((j & 1) == 0)
          nib[j >> 1] = (uint8_t)v;  // high nibble: next value, or zero padding
        else
          nib[j >> 1] = (uint8_t)((nib[j >> 1] & 0x0Fu) | v << 4);
      }
    }
    if (WITH_FLAGS) flags[g] = (uint8_t)fl;
  }
  if (WITH_STATS) flush_stats2(stats, bits, unc);
}

// ---- Hamming(8,4) with packed values / error types ---------------------------

// 4 data bytes (0x0d each) -> 16 bits d0 | d1 << 4 | d2 << 8 | d3 << 12
__device__ __forceinline__ uint32_t nib_pack4(uint32_t w) {
  const uint32_t x = w | (w >> 4);  // byte0 = d0|d1<<4, byte2 = d2|d3<<4
  return (x & 0xFFu) | ((x >> 8) & 0xFF00u);
}
// 16 bits of 4 nibbles -> 4 bytes (0x0d each)
__device__ __forceinline__ uint32_t nib_unpack4(uint32_t h) {
  const uint32_t x = (h & 0xFFu) | (h & 0xFF00u) << 8;  // byte0 = d0|d1<<4, byte2 = d2|d3<<4
  return (x & 0x000F000Fu) | (x << 4 & 0x0F000F00u);
}
// 4 type bytes (0..3) -> 8 bits t0 | t1 << 2 | t2 << 4 | t3 << 6
__device__ __forceinline__ uint32_t type_pack4(uint32_t t) {
  const uint32_t x = t | (t >> 6);          // byte0 = t0|t1<<2, byte2 = t2|t3<<2
  return (x & 0xFu) | ((x >> 12) & 0xF0u);
}

constexpr int kHpBlock = 256;

// a lane owns 16 values: one 16-byte codeword access, 8 bytes of nibbles.
// Grid-stride at 64 workgroups per CU (kHpEncPerCu): 32.4-33.1 us against
// 33.6-33.8 at 32, and at or within noise of full grids with 1, 2 or 4 chunks
// per lane (34.3 / 32.6 / 34.7) at config 2's 134 M values
// (profiles/r06/h84_packed_encode_grid.txt, tools/exp/h84_pk_enc_exp.hip)
constexpr int kHpEncPerCu = 64;
__global__ __launch_bounds__(kHpBlock) void h84_encode_packed_kernel(const u32x2 *__restrict__ nib,
                                                                     u32x4 *__restrict__ cw,
                                                                     int64_t n16) {
  for (int64_t i = (int64_t)blockIdx.x * kHpBlock + threadIdx.x; i < n16;
       i += (int64_t)gridDim.x * kHpBlock) {
    const u32x2 v = ld_stream(nib + i);
    u32x4 o;
    o.x = h84_encode4(nib_unpack4(v.x & 0xFFFFu));
    o.y = h84_encode4(nib_unpack4(v.x >> 16));
    o.z = h84_encode4(nib_unpack4(v.y & 0xFFFFu));
    o.w = h84_encode4(nib_unpack4(v.y >> 16));
    st_stream(cw + i, o);
  }
}

// 16 values per lane.  The packing works on pairs of words with v_perm, and the
// statistics come from the packed ErrorType word (2 bits per value: 1 =
// corrected single, 2 = double) instead of per-word popcounts: ~25 % fewer VALU
// ops than packing and counting word by word, which the counters showed this
// kernel spending most of its time on.  Grid-stride, 32 workgroups per CU: 16 /
// 64 / 128 per CU, two chunks' loads in flight per lane, and persistent 4-chunk
// wave tiles with the dynamic tail all measured slower (43.4-52.7 and 48.2 us
// against 41.9; profiles/r03/packed/h84_packed_grid_unroll_ab.log).
constexpr int kHpGridPerCu = 32;
template <bool WITH_TYPES, bool WITH_STATS>
__global__ __launch_bounds__(kHpBlock) void h84_decode_packed_kernel(const u32x4 *__restrict__ cw,
                                                                     u32x2 *__restrict__ nib,
                                                                     uint32_t *__restrict__ types,
                                                                     int64_t n16,
                                                                     uint64_t *__restrict__ stats) {
  uint32_t n1 = 0, n2 = 0;
  auto chunk = [&](const u32x4 c, int64_t i) {
    const uint32_t w[4] = {c.x, c.y, c.z, c.w};
    uint32_t y[4], z[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const HammingTables tb(w[k]);
      const uint32_t d = (w[k] ^ (tb.fx & tb.pe_rep)) & 0x0F0F0F0Fu;  // correct only SINGLE (pe && nz)
      const uint32_t pe = tb.pe(), nz = tb.nz();
      const uint32_t t = pe | (pe ^ nz) << 1;  // per byte, hamming84_triton.py:185-187
      y[k] = d | d >> 4;  // bytes 0 and 2: (v0 | v1 << 4), (v2 | v3 << 4)
      z[k] = t | t >> 6;  // bytes 0 and 2: (t0 | t1 << 2), (t2 | t3 << 2)
    }
    // bytes 0 and 2 of each word, two words per v_perm
    const uint32_t n01 = __builtin_amdgcn_perm(y[1], y[0], 0x06040200u);
    const uint32_t n23 = __builtin_amdgcn_perm(y[3], y[2], 0x06040200u);
    st_stream(nib + i, u32x2{n01, n23});
    if (WITH_TYPES || WITH_STATS) {
      uint32_t r01 = __builtin_amdgcn_perm(z[1], z[0], 0x06040200u);  // 4-bit fields, one per byte
      uint32_t r23 = __builtin_amdgcn_perm(z[3], z[2], 0x06040200u);
      r01 |= r01 >> 4;
      r23 |= r23 >> 4;
      const uint32_t tw = __builtin_amdgcn_perm(r23, r01, 0x06040200u);  // 16 x 2 bits, value j at 2j
      if (WITH_TYPES) st_stream(types + i, tw);
      if (WITH_STATS) {
        const uint32_t hi = tw >> 1;
        n1 += __builtin_popcount(tw & ~hi & 0x55555555u);  // type 1: single, corrected
        n2 += __builtin_popcount(hi & ~tw & 0x55555555u);  // type 2: double, detected
      }
    }
  };
  const int64_t stride = (int64_t)gridDim.x * kHpBlock;
  int64_t i = (int64_t)blockIdx.x * kHpBlock + threadIdx.x;
  for (; i < n16; i += stride) chunk(ld_stream(cw + i), i);
  if (WITH_STATS) flush_stats2<kHpBlock>(stats, n1, n2);
}

// tails and unaligned buffers, byte accesses: encode one thread per value,
// decode one thread per group of 4 values (2 nibble bytes + 1 type byte, never
// shared because `begin` is a multiple of 16)
__global__ __launch_bounds__(kBlock) void h84_encode_packed_tail_kernel(const uint8_t *__restrict__ nib,
                                                                        uint8_t *__restrict__ cw,
                                                                        int64_t begin, int64_t n) {
  for (int64_t j = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n;
       j += (int64_t)gridDim.x * kBlock)
    cw[j] = (uint8_t)(h84_encode4(nib[j >> 1] >> (4 * (j & 1)) & 0xFu) & 0xFFu);
}

__global__ __launch_bounds__(kBlock) void h84_decode_packed_tail_kernel(
    const uint8_t *__restrict__ cw, uint8_t *__restrict__ nib, uint8_t *__restrict__ types,
    int64_t begin, int64_t n, uint64_t *__restrict__ stats) {
  uint32_t n1 = 0, n2 = 0;
  for (int64_t g = begin / 4 + (int64_t)blockIdx.x * kBlock + threadIdx.x; g * 4 < n;
       g += (int64_t)gridDim.x * kBlock) {
    uint32_t tb = 0, nb[2] = {0, 0};
    for (int64_t j = 4 * g; j < n && j < 4 * g + 4; ++j) {
      uint32_t d, t;
      h84_decode4(cw[j], d, t, n1, n2);
      nb[(j >> 1) & 1] |= d << (4 * (j & 1));
      tb |= t << (2 * (j & 3));
    }
    nib[2 * g] = (uint8_t)nb[0];
    if (4 * g + 2 < n) nib[2 * g + 1] = (uint8_t)nb[1];
    if (types) types[g] = (uint8_t)tb;
  }
  if (stats) flush_stats2(stats, n1, n2);
}
}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_golay_encode_packed(const uint8_t *nibbles, uint8_t *codewords, int64_t m,
                                        void *stream) {
  if (m < 0) return set_error(KVECC_EINVAL, "golay_encode_packed: negative m");
  if (m == 0) return KVECC_OK;
  if (!nibbles || !codewords) return set_error(KVECC_EINVAL, "golay_encode_packed: null pointer");
  const uint16_t *par = golay_parity_table_dev();
  if (!par) return KVECC_EHIP;
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (aligned(nibbles, 4) && aligned(codewords, 4)) {
    const int64_t ntiles = m / kPkTile;
    if (ntiles > 0)
      KVECC_LAUNCH(golay_encode_packed_kernel, dim3(grid_for(ntiles, 1, 16)), dim3(kPkBlock), 0,
                         st, reinterpret_cast<const uint32_t *>(nibbles),
                         reinterpret_cast<uint32_t *>(codewords), ntiles, par);
    done = ntiles * kPkTile;
  }
  if (done < m)
    KVECC_LAUNCH(golay_encode_packed_tail_kernel, dim3((unsigned)cdiv(m - done, kBlock)),
                       dim3(kBlock), 0, st, nibbles, codewords, done, m, par);
  return check_launch("golay_encode_packed");
}

KVECC_API int kvecc_golay_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                        uint8_t *uncorrectable, int64_t m, uint64_t *stats,
                                        void *stream) {
  if (m < 0) return set_error(KVECC_EINVAL, "golay_decode_packed: negative m");
  if (m == 0) return KVECC_OK;
  if (!nibbles || !codewords) return set_error(KVECC_EINVAL, "golay_decode_packed: null pointer");
  const uint16_t *par = golay_parity_table_dev(), *cor = golay_correct_table_dev();
  if (!par || !cor) return KVECC_EHIP;
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  const int64_t wave_tiles = m / kPk2TileCw;
  if (aligned(nibbles, 4) && aligned(codewords, 16) && wave_tiles > 0 &&
      wave_tiles * kPk2TileBytes < ((int64_t)1 << 31)) {
    const uint8_t *tab = golay_pk_table_dev();
    uint32_t *dyn = shim_dyn_slot(stream);
    if (!tab || !dyn) return KVECC_EHIP;
    const PkDecArgs a{codewords, reinterpret_cast<uint32_t *>(nibbles), uncorrectable, (uint32_t)wave_tiles,
                      tab, stats, dyn};
    const dim3 grid(grid_for(wave_tiles, kPk2Waves, kPk2PerCu)), block(kPk2Block);
    if (uncorrectable && stats)
      KVECC_LAUNCH((golay_decode_packed_wave_kernel<true, true>), grid, block, 0, st, a);
    else if (uncorrectable)
      KVECC_LAUNCH((golay_decode_packed_wave_kernel<true, false>), grid, block, 0, st, a);
    else if (stats)
      KVECC_LAUNCH((golay_decode_packed_wave_kernel<false, true>), grid, block, 0, st, a);
    else
      KVECC_LAUNCH((golay_decode_packed_wave_kernel<false, false>), grid, block, 0, st, a);
    done = wave_tiles * kPk2TileCw;
  } else if (aligned(nibbles, 4) && aligned(codewords, 16)) {
    const int64_t ntiles = m / kPkTile;
    if (ntiles > 0) {
      const dim3 grid(grid_for(ntiles, 1, kPkDecPerCu)), block(kPkBlock);
      const uint32_t *c = reinterpret_cast<const uint32_t *>(codewords);
      uint32_t *n = reinterpret_cast<uint32_t *>(nibbles);
      if (uncorrectable && stats)
        KVECC_LAUNCH((golay_decode_packed_staged_kernel<true, true>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
      else if (uncorrectable)
        KVECC_LAUNCH((golay_decode_packed_staged_kernel<true, false>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
      else if (stats)
        KVECC_LAUNCH((golay_decode_packed_staged_kernel<false, true>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
      else
        KVECC_LAUNCH((golay_decode_packed_staged_kernel<false, false>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
    }
    done = ntiles * kPkTile;
  } else if (aligned(nibbles, 4) && aligned(codewords, 4)) {
    const int64_t ntiles = m / kPkTile;
    if (ntiles > 0) {
      const dim3 grid(grid_for(ntiles, 1, 32)), block(kPkBlock);
      const uint32_t *c = reinterpret_cast<const uint32_t *>(codewords);
      uint32_t *n = reinterpret_cast<uint32_t *>(nibbles);
      if (uncorrectable && stats)
        KVECC_LAUNCH((golay_decode_packed_kernel<true, true>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
      else if (uncorrectable)
        KVECC_LAUNCH((golay_decode_packed_kernel<true, false>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
      else if (stats)
        KVECC_LAUNCH((golay_decode_packed_kernel<false, true>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
      else
        KVECC_LAUNCH((golay_decode_packed_kernel<false, false>), grid, block, 0, st, c, n, uncorrectable, ntiles, par, cor, stats);
    }
    done = ntiles * kPkTile;
  }
  if (done < m) {
    const dim3 grid(grid_for(cdiv(m - done, 8), kBlock)), block(kBlock);
    if (uncorrectable && stats)
      KVECC_LAUNCH((golay_decode_packed_tail_kernel<true, true>), grid, block, 0, st, codewords, nibbles, uncorrectable, done, m, par, cor, stats);
    else if (uncorrectable)
      KVECC_LAUNCH((golay_decode_packed_tail_kernel<true, false>), grid, block, 0, st, codewords, nibbles, uncorrectable, done, m, par, cor, stats);
    else if (stats)
      KVECC_LAUNCH((golay_decode_packed_tail_kernel<false, true>), grid, block, 0, st, codewords, nibbles, uncorrectable, done, m, par, cor, stats);
    else
      KVECC_LAUNCH((golay_decode_packed_tail_kernel<false, false>), grid, block, 0, st, codewords, nibbles, uncorrectable, done, m, par, cor, stats);
  }
  return check_launch("golay_decode_packed");
}

KVECC_API int kvecc_hamming84_encode_packed(const uint8_t *nibbles, uint8_t *codewords, int64_t n,
                                            void *stream) {
  if (n < 0) return set_error(KVECC_EINVAL, "hamming84_encode_packed: negative n");
  if (n == 0) return KVECC_OK;
  if (!nibbles || !codewords) return set_error(KVECC_EINVAL, "hamming84_encode_packed: null pointer");
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (aligned(nibbles, 8) && aligned(codewords, 16)) {
    const int64_t n16 = n / 16;
    if (n16 > 0)
      KVECC_LAUNCH(h84_encode_packed_kernel, dim3(grid_for(n16, kHpBlock, kHpEncPerCu)), dim3(kHpBlock),
                         0, st, reinterpret_cast<const u32x2 *>(nibbles),
                         reinterpret_cast<u32x4 *>(codewords), n16);
    done = n16 * 16;
  }
  if (done < n)
    KVECC_LAUNCH(h84_encode_packed_tail_kernel, dim3(grid_for(n - done, kBlock)), dim3(kBlock),
                       0, st, nibbles, codewords, done, n);
  return check_launch("hamming84_encode_packed");
}

KVECC_API int kvecc_hamming84_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                            uint8_t *error_types, int64_t n, uint64_t *stats,
                                            void *stream) {
  if (n < 0) return set_error(KVECC_EINVAL, "hamming84_decode_packed: negative n");
  if (n == 0) return KVECC_OK;
  if (!nibbles || !codewords) return set_error(KVECC_EINVAL, "hamming84_decode_packed: null pointer");
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (done < n && aligned(nibbles, 8) && aligned(codewords, 16) && (!error_types || aligned(error_types, 4))) {
    const int64_t n16 = (n - done) / 16;
    if (n16 > 0) {
      const dim3 grid(grid_for(n16, kHpBlock, kHpGridPerCu)), block(kHpBlock);
      const int64_t i0 = done / 16;
      const u32x4 *c = reinterpret_cast<const u32x4 *>(codewords) + i0;
      u32x2 *o = reinterpret_cast<u32x2 *>(nibbles) + i0;
      uint32_t *t = error_types ? reinterpret_cast<uint32_t *>(error_types) + i0 : nullptr;
      if (error_types && stats)
        KVECC_LAUNCH((h84_decode_packed_kernel<true, true>), grid, block, 0, st, c, o, t, n16, stats);
      else if (error_types)
        KVECC_LAUNCH((h84_decode_packed_kernel<true, false>), grid, block, 0, st, c, o, t, n16, stats);
      else if (stats)
        KVECC_LAUNCH((h84_decode_packed_kernel<false, true>), grid, block, 0, st, c, o, t, n16, stats);
      else
        KVECC_LAUNCH((h84_decode_packed_kernel<false, false>), grid, block, 0, st, c, o, t, n16, stats);
    }
    done += n16 * 16;
  }
  if (done < n)
    KVECC_LAUNCH(h84_decode_packed_tail_kernel, dim3(grid_for(cdiv(n - done, 4), kBlock)),
                       dim3(kBlock), 0, st, codewords, nibbles, error_types, done, n, stats);
  return check_launch("hamming84_decode_packed");
}

}  // extern "C"
