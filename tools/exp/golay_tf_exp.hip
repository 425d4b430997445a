// golay_tf_exp.hip -- the fused Golay read on a FULL grid (one wave tile per
// wave, as the byte-codec reads) with a table-free error path, NOT shipped.
// Built with the product sources (#includes shim.hip for the tile helpers)
// into tools/exp/libgtf.so; tools/exp/run_golay_tf_exp.py times it against the
// product's persistent kernel and compares outputs and statistics.
//
// Why: the persistent read (160 us) stages 32 KiB of tables once per
// workgroup; a full grid has 16 K workgroups, and staging even the 8 KiB
// uint16 tables per workgroup cost more than the full grid saved
// (profiles/r04/fused/read_exp_ab_*.log).  Here a workgroup stages only the
// parity half as two 64-entry tables (512 B): p(d) = T[d & 63] ^ T[64 + (d >> 6)]
// (spread data | parity << 20, linear in d).  The correction needs no table:
// B is symmetric with B B = I (runtime.hip kGolayRow), so for s = e_d B ^ e_p
//   wt(s) <= 3                       -> e = (0, s)
//   u = s B, wt(u) <= 3               -> e = (u, 0)
//   wt(s ^ B_i) <= 2 for some i        -> e = (unit_i, s ^ B_i)
//   wt(u ^ B_j) <= 2 for some j        -> e = (u ^ B_j, unit_j)
//   otherwise                          -> uncorrectable (weight >= 4)
// which is the unique coset leader of weight <= 3, i.e. exactly the
// reference's 4096-entry table (golay_triton.py:213-295; checked on every
// syndrome by tests/test_golay_table_free.py).
// Nonzero syndromes (~21 % of codewords at BER 1e-2) are queued per wave in LDS
// (ballot + mbcnt) and decoded 64 at a time ("fast" rounds: the first two
// tests, ~25 operations); the mixed-weight ones (~6 % of those) go to a second
// queue for the 24 weight tests ("slow" rounds).  Corrections are XORed into
// the wave's staged tile (ds_xor), which phase 2 dequantizes as the product.
//
// VAR 0: the decoder above; 1: syndromes only, no queues (WRONG values: the
// cost of the error path); 2: fast rounds only (WRONG on mixed errors);
// 3: the queued syndromes' corrections gathered from the global 16 KiB
// correction table (L2-resident), 4 rounds of gathers in flight.
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/shim.hip"

namespace kvecc {
namespace exp {

// one LDS queue per wave: nonzero syndromes, then (written over the consumed
// entries) the mixed-weight ones; drained at the end of phase 1, or before a
// group that could overflow it (> kQ - 256 queued: BER >~ 3e-2)
constexpr int kQ = 512;
constexpr uint32_t kRowB[12] = {0xA3B, 0xD1D, 0xE8E, 0xB47, 0xDA3, 0xED1,
                                0xF68, 0xBB4, 0x9DA, 0x8ED, 0xC76, 0x7FF};

__device__ __forceinline__ uint32_t tf_par(const uint32_t *ptab, uint32_t x) {
  return ptab[x & 63u] ^ ptab[64u + ((x >> 6) & 63u)];
}

// XOR a spread correction (nibbles in bytes 0-2) into the 3 staged bytes at o
__device__ __forceinline__ void tf_xor(uint8_t *stage, uint32_t o, uint32_t c) {
  const uint32_t sh = (o & 3u) * 8u;
  uint32_t *p = reinterpret_cast<uint32_t *>(stage + (o & ~3u));
  __hip_atomic_fetch_xor(p, c << sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  if (sh >= 16u) __hip_atomic_fetch_xor(p + 1, c >> (32u - sh), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__device__ __forceinline__ uint32_t tf_spread(uint32_t x) {
  return (x & 0xFu) | (x & 0xF0u) << 4 | (x & 0xF00u) << 8;
}

__device__ __forceinline__ uint32_t lane_prefix(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

template <bool PACKED, int VAR>
__global__ __launch_bounds__(kTileBlock) void golay_tf_kernel(ShimTileArgs a) {
  using TO = __half;
  __shared__ uint32_t ptab[128];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kTileWaves][kTileStage];
  __shared__ float scale_all[kTileWaves][kWave];
  __shared__ uint32_t q_all[kTileWaves][kQ];
  if (threadIdx.x < 128) ptab[threadIdx.x] = a.atab[threadIdx.x < 64 ? threadIdx.x : (threadIdx.x - 64) << 6];
  __syncthreads();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const uint32_t lane = threadIdx.x % kWave;
  const uint32_t gw = blockIdx.x * kTileWaves + wave;
  if (gw >= a.units) return;
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
  const ShimTile t = shim_tile(a, gw);
  u32x4 w[kTileGroups];
  float scale;
  tile_issue<PACKED>(a, t, lane, it, w, scale);
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const uint32_t v = lane + kWave * i;
    const uint32_t r = v / dv, j = v - r * dv;
    it.r2[i] = min(r, a.tr - 1);
    it.j2[i] = it.r2[i] * a.lr + V * j;
    it.o2[i] = (r * a.d + V * j) * (uint32_t)sizeof(TO);
  }
  uint8_t *stage = stage_all[wave];
  uint32_t *fq = q_all[wave];
  uint32_t fq_n = 0;  // wave-uniform
  uint32_t bits = 0, unc = 0;
  scale_all[wave][lane] = scale;

  // the 24 weight tests of the mixed-weight syndromes fq[0, cnt)
  auto slow_round = [&](uint32_t base, uint32_t cnt) {
    const bool on = lane < cnt;
    const uint32_t e = on ? fq[base + lane] : 0u;
    const uint32_t s = e & 0xFFFu, o = e >> 12;
    const uint32_t u = tf_par(ptab, s) >> 20;
    uint32_t ks = ~0u, ku = ~0u;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const uint32_t ts = s ^ kRowB[i], tu = u ^ kRowB[i];
      ks = min(ks, (uint32_t)__builtin_popcount(ts) << 4 | (uint32_t)i);
      ku = min(ku, (uint32_t)__builtin_popcount(tu) << 12 | tu);
    }
    uint32_t ed = 0, n = 4;
    if ((ks >> 4) <= 2u) {
      ed = 1u << (ks & 15u);
      n = 1u + (ks >> 4);
    } else if ((ku >> 12) <= 2u) {
      ed = ku & 0xFFFu;
      n = 1u + (ku >> 12);
    }
    if (on) {
      if (ed) tf_xor(stage, o, tf_spread(ed));
      if (n == 4u) ++unc;
      else bits += n;
    }
  };
  // every queued syndrome: the two cheap tests, 64 per round; the mixed-weight
  // ones are rewritten to the queue's front (never past the entries already
  // read), then decoded by slow rounds
  auto drain = [&]() {
    wave_lds_sync();
    if (VAR == 3) {  // correction entries from the global table, 4 rounds' gathers in flight
      const uint32_t *cor = a.atab + 4096;
      for (uint32_t base = 0; base < fq_n; base += 4 * kWave) {
        uint32_t e[4], c[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const bool on = base + k * kWave + lane < fq_n;
          e[k] = on ? fq[base + k * kWave + lane] : 0u;
          c[k] = on ? cor[e[k] & 0xFFFu] : 0u;
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (c[k] & 0x000F0F0Fu) tf_xor(stage, e[k] >> 12, c[k] & 0x000F0F0Fu);
          bits += (c[k] >> 24) & 63u;
          unc += c[k] >> 30;
        }
      }
      fq_n = 0;
      return;
    }
    uint32_t sq_n = 0;
    for (uint32_t base = 0; base < fq_n; base += kWave) {
      const uint32_t cnt = min(fq_n - base, (uint32_t)kWave);
      const bool on = lane < cnt;
      const uint32_t e = on ? fq[base + lane] : 0u;
      const uint32_t s = e & 0xFFFu, o = e >> 12;
      const uint32_t ws = __builtin_popcount(s);
      const uint32_t pu = tf_par(ptab, s);
      const uint32_t u = pu >> 20;
      const uint32_t wu = __builtin_popcount(u);
      const bool slow = on && ws > 3u && wu > 3u;
      if (on && ws > 3u && wu <= 3u) tf_xor(stage, o, tf_spread(u));
      if (on && !slow) bits += ws <= 3u ? ws : wu;
      if (VAR == 2) continue;
      const uint64_t m = __ballot(slow);
      wave_lds_sync();  // this round's entries are read
      if (slow) fq[sq_n + lane_prefix(m)] = e;
      sq_n += (uint32_t)__builtin_popcountll(m);
    }
    if (VAR == 0 && sq_n) {
      wave_lds_sync();
      for (uint32_t base = 0; base < sq_n; base += kWave) slow_round(base, min(sq_n - base, (uint32_t)kWave));
    }
    fq_n = 0;
  };

  // ---- phase 1: syndromes, staged data, queued errors --------------------------
#pragma unroll
  for (int i = 0; i < kTileGroups; ++i) {
    if (i * kWave >= (int)groups) break;  // uniform
    if (VAR != 1 && i >= 2 && fq_n > (uint32_t)(kQ - kTileGroups * kWave)) drain();  // uniform, rare
    const uint32_t q = it.q1[i], r = it.r1[i];
    const uint32_t obase = r * a.lr + 12u * q;
    uint32_t sp[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t cw = tile_cw<PACKED>(w[i], c);
      if (c > 0) cw = 4 * q + c < a.g ? cw : 0u;
      const uint32_t p = tf_par(ptab, cw);
      const uint32_t s = ((cw >> 12) ^ (p >> 20)) & 0xFFFu;
      sp[c] = p & 0x000F0F0Fu;
      if (VAR == 1) {
        bits += s != 0u;
        continue;
      }
      const bool flag = s != 0u;
      const uint64_t m = __ballot(flag);
      if (flag) fq[fq_n + lane_prefix(m)] = s | (obase + 3u * c) << 12;
      fq_n += (uint32_t)__builtin_popcountll(m);
    }
    if (r < a.tr) {
      uint32_t *dst = reinterpret_cast<uint32_t *>(stage + obase);
      dst[0] = sp[0] | sp[1] << 24;
      dst[1] = sp[1] >> 8 | sp[2] << 16;
      dst[2] = sp[2] >> 16 | sp[3] << 8;
    }
  }
  if (VAR != 1) drain();
  wave_lds_sync();
  // ---- phase 2: dequantize, one 16-byte store per lane per item (as the product)
  const __amdgpu_buffer_rsrc_t os = tile_out<TO>(a, t);
  const bool dead = t.row0 < 0;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    if (i * kWave >= (int)chunks) break;  // uniform
    const uint32_t *src = reinterpret_cast<const uint32_t *>(stage + it.j2[i]);
    const uint32_t nb[2] = {src[0], src[1]};
    tile_store(os, it.o2[i], dq16<TO>(nb, scale_all[wave][it.r2[i]], dead));
  }
  bits = wave_sum(bits);
  unc = wave_sum(unc);
  if (lane == 0) {
    uint64_t *slot = a.stats + (gw % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (bits) atomicAdd(reinterpret_cast<unsigned long long *>(slot), (unsigned long long)bits);
    if (unc) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), (unsigned long long)unc);
  }
}

struct Variant {
  const char *name;
  void (*kern)(ShimTileArgs);
};

const Variant kVariants[] = {
    {"tf", golay_tf_kernel<false, 0>},
    {"tf_synonly", golay_tf_kernel<false, 1>},
    {"tf_fastonly", golay_tf_kernel<false, 2>},
    {"pk_tf", golay_tf_kernel<true, 0>},
    {"pk_tf_synonly", golay_tf_kernel<true, 1>},
    {"gq", golay_tf_kernel<false, 3>},
    {"pk_gq", golay_tf_kernel<true, 3>},
};

}  // namespace exp
}  // namespace kvecc

extern "C" {

__attribute__((visibility("default"))) int kvecc_exp_gtf_count(void) {
  return (int)(sizeof(kvecc::exp::kVariants) / sizeof(kvecc::exp::kVariants[0]));
}

__attribute__((visibility("default"))) const char *kvecc_exp_gtf_name(int v) { return kvecc::exp::kVariants[v].name; }

// the fused Golay read of shim_read_batch (fp16 out, statistics on) through
// variant v on a full grid; lds_pad: dynamic LDS bytes (caps workgroups per CU)
__attribute__((visibility("default"))) int kvecc_exp_gtf(int v, const void *k_cache, const void *v_cache,
                                                        const float *k_scales, const float *v_scales,
                                                        const int32_t *table, int64_t tstride, int64_t batch,
                                                        int64_t ctx, int64_t hkv, int64_t d, int64_t block_size,
                                                        int packed, void *k_out, void *v_out, uint64_t *stats,
                                                        int lds_pad, void *stream) {
  using namespace kvecc;
  if (d % 8 != 0) return KVECC_EINVAL;
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
  // queue offsets are 12 bits: every staged byte offset must be < 4096
  if (a.tr * a.lr > 4096) return KVECC_EINVAL;
  const unsigned grid = (unsigned)cdiv(a.units, kTileWaves);
  KVECC_LAUNCH(exp::kVariants[v].kern, dim3(grid), dim3(kTileBlock), (unsigned)lds_pad, as_stream(stream), a);
  return check_launch("exp_gtf");
}

}  // extern "C"
