// packed_dec_exp.hip -- experimental variants of the packed Golay decode
// (csrc/packed.hip golay_decode_packed_wave_kernel), NOT shipped: this file
// #includes packed.hip for its helpers; tools/exp/run_packed_dec_exp.py times
// the variants against the product in one process.
//   GATHER 0: the real table lookups; 1: lane-private, conflict-free addresses
//          (same instruction count, WRONG values: do the LDS bank conflicts
//          cost time?)
//   GLDS   the tile's codeword bytes go to LDS by LDS-DMA (global_load_lds,
//          double-buffered stage, no VGPR round trip and no ds_write)
//   BLOCK, PCT: workgroup size, static share of the dynamic tail
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/packed.hip"

namespace kvecc {
namespace exp {

template <int GATHER, bool GLDS, int BLOCK, int PCT>
__global__ __launch_bounds__(BLOCK) void pkdec_exp_kernel(PkDecArgs a) {
  constexpr int kW = BLOCK / kWave;
  constexpr int kStages = GLDS ? 2 : 1;
  __shared__ __attribute__((aligned(16))) uint8_t tab[24576];
  __shared__ __attribute__((aligned(16))) uint8_t stage_all[kW][kStages][kPk2TileBytes];
  for (int i = threadIdx.x; i < 24576 / 16; i += BLOCK)
    reinterpret_cast<u32x4 *>(tab)[i] = reinterpret_cast<const u32x4 *>(a.tab)[i];
  __syncthreads();
  const uint32_t wave = uni((uint32_t)threadIdx.x / kWave), lane = threadIdx.x % kWave;
  const uint32_t gw = blockIdx.x * kW + wave, nwaves = gridDim.x * kW;
  if (gw >= a.units) return;
  TileSchedule sched;
  sched.init(a.units, a.dyn, gw, nwaves, lane, PCT);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t *>(a.cw), 0, (int)(a.units * (uint32_t)kPk2TileBytes), 0x00020000);
  uint32_t t = gw;
  u32x4 nxt[kPk2Vec];
  uint32_t sb = 0;  // GLDS: the stage buffer holding tile t
  auto issue = [&](uint32_t tt, uint32_t buf) {
    if (GLDS) {
      const uint8_t *src = a.cw + (size_t)tt * kPk2TileBytes;
#pragma unroll
      for (int k = 0; k < kPk2Vec; ++k)
        __builtin_amdgcn_global_load_lds(
            reinterpret_cast<const void *>(src + 16u * (lane + kWave * k)),
            reinterpret_cast<__attribute__((address_space(3))) void *>(
                reinterpret_cast<uintptr_t>(&stage_all[wave][buf][0]) + 1024 * k),
            16, 0, 0);
    } else {
#pragma unroll
      for (int k = 0; k < kPk2Vec; ++k)
        nxt[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                               rs, tt * (uint32_t)kPk2TileBytes + 16u * (lane + kWave * k), 0, 2));
    }
  };
  issue(t, 0);
  uint32_t bits = 0, unc = 0;
  for (;;) {
    uint8_t *stage = stage_all[wave][sb];
    if (GLDS) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
#pragma unroll
      for (int k = 0; k < kPk2Vec; ++k) reinterpret_cast<u32x4 *>(stage)[lane + kWave * k] = nxt[k];
    }
    wave_lds_sync();
    const uint32_t cur = t;
    t = sched.next(t, lane);
    const bool more = t < a.units;
    if (more) issue(t, sb ^ 1u);
#pragma unroll
    for (int g = 0; g < kPk2Groups; ++g) {
      const u32x2 *p = reinterpret_cast<const u32x2 *>(stage + (g * kWave + lane) * 24);
      const u32x2 x0 = p[0], x1 = p[1], x2 = p[2];
      const uint32_t w[6] = {x0.x, x0.y, x1.x, x1.y, x2.x, x2.y};
      uint32_t c[8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        c[4 * h] = w[3 * h];
        c[4 * h + 1] = __builtin_amdgcn_alignbyte(w[3 * h + 1], w[3 * h], 3);
        c[4 * h + 2] = __builtin_amdgcn_alignbyte(w[3 * h + 2], w[3 * h + 1], 2);
        c[4 * h + 3] = w[3 * h + 2] >> 8;
      }
      uint32_t d[8], esum = 0, fl = 0;
#pragma unroll
      for (int k = 7; k >= 0; --k) {
        uint32_t pv, e;
        if (GATHER == 1) {  // bank = lane % 32, data-dependent row: conflict-free, wrong values
          pv = *reinterpret_cast<const uint32_t *>(tab + 4 * ((lane & 31u) + 32u * (c[k] & 63u)));
          e = *reinterpret_cast<const uint32_t *>(tab + 8192 + 4 * ((lane & 31u) + 32u * ((c[k] ^ pv) >> 12 & 127u)));
        } else {
          pv = *reinterpret_cast<const uint16_t *>(tab + ((c[k] << 1) & 0x1FFEu));
          const uint32_t off = __builtin_amdgcn_bitop3_b32(c[k] >> 10, pv, 0x3FFCu, 0x28);
          e = *reinterpret_cast<const uint32_t *>(tab + 8192 + off);
        }
        d[k] = __builtin_amdgcn_bitop3_b32(c[k], e, 0xFFFu, 0x28);
        esum += e;
        fl = __builtin_amdgcn_alignbit(fl, e, 31);
      }
      bits += (esum >> 24) & 0x7Fu;
      unc += __builtin_popcount(fl);
      uint32_t n[3];
      nib_pack8(d, n);
      const uint32_t grp = cur * (kPk2TileCw / 8) + g * kWave + lane;
      st_stream(reinterpret_cast<u32x3v *>(a.nib + (size_t)grp * 3), u32x3v{n[0], n[1], n[2]});
      st_stream(a.flags + grp, (uint8_t)fl);
    }
    if (!more) break;
    wave_lds_sync();
    if (GLDS) sb ^= 1u;
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
  void (*kern)(PkDecArgs);
  int block;
};
static const Variant kVariants[] = {
    {"pk", pkdec_exp_kernel<0, false, 512, 75>, 512},
    {"pk_cfree", pkdec_exp_kernel<1, false, 512, 75>, 512},
    {"pk_glds", pkdec_exp_kernel<0, true, 512, 75>, 512},
    {"pk_b256", pkdec_exp_kernel<0, false, 256, 75>, 256},
    {"pk_glds_b256", pkdec_exp_kernel<0, true, 256, 75>, 256},
    {"pk_p50", pkdec_exp_kernel<0, false, 512, 50>, 512},
    {"pk_p90", pkdec_exp_kernel<0, false, 512, 90>, 512},
    {"pk_cfree_glds", pkdec_exp_kernel<1, true, 512, 75>, 512},
    {"pk_p60", pkdec_exp_kernel<0, false, 512, 60>, 512},
    {"pk_p65", pkdec_exp_kernel<0, false, 512, 65>, 512},
    {"pk_p85", pkdec_exp_kernel<0, false, 512, 85>, 512},
    {"pk_p40", pkdec_exp_kernel<0, false, 512, 40>, 512},
    {"pk_b256_p50", pkdec_exp_kernel<0, false, 256, 50>, 256},
    {"pk_b384", pkdec_exp_kernel<0, false, 384, 75>, 384},
    {"pk_b384_p50", pkdec_exp_kernel<0, false, 384, 50>, 384},
    {"pk_b256_p30", pkdec_exp_kernel<0, false, 256, 30>, 256},
    {"pk_b256_p40", pkdec_exp_kernel<0, false, 256, 40>, 256},
    {"pk_b256_p20", pkdec_exp_kernel<0, false, 256, 20>, 256},
    {"pk_p30", pkdec_exp_kernel<0, false, 512, 30>, 512},
};

}  // namespace exp
}  // namespace kvecc

extern "C" {
__attribute__((visibility("default"))) int kvecc_exp_pkdec_count(void) {
  return (int)(sizeof(kvecc::exp::kVariants) / sizeof(kvecc::exp::kVariants[0]));
}
__attribute__((visibility("default"))) const char *kvecc_exp_pkdec_name(int v) { return kvecc::exp::kVariants[v].name; }
// m must be a multiple of the 1024-codeword wave tile; flags and stats required
__attribute__((visibility("default"))) int kvecc_exp_pkdec(int v, const uint8_t *cw, uint8_t *nib, uint8_t *flags,
                                                          int64_t m, uint64_t *stats, int per_cu, void *stream) {
  using namespace kvecc;
  if (m % kPk2TileCw) return set_error(KVECC_EINVAL, "exp_pkdec: m %% tile");
  const exp::Variant &var = exp::kVariants[v];
  PkDecArgs a{cw, reinterpret_cast<uint32_t *>(nib), flags, (uint32_t)(m / kPk2TileCw), golay_pk_table_dev(), stats,
              shim_dyn_slot(stream)};
  const unsigned grid = grid_for(a.units, var.block / kWave, per_cu);
  KVECC_LAUNCH(var.kern, dim3(grid), dim3(var.block), 0, as_stream(stream), a);
  return check_launch("exp_pkdec");
}
}
