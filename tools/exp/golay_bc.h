// golay_bc.h -- the byte-class Golay(24,12) decoder's tables (experiments
// only: tools/exp/golay_read_exp.hip, golay_dec_exp.hip).  Include inside
// namespace kvecc::exp after codec_math.h.
#pragma once

#include <vector>

namespace kvecc {
namespace exp {

// Byte-class Golay decoder (GATHER 5).  With the systematic generator [I | B]
// (B symmetric, B B = I) an error (de, pe) of weight <= 3 has syndrome
// s = B de ^ pe, and q = B s = de ^ B pe.  Either wt(pe) <= 1 and de = B (s ^ m)
// with m = pe's data-side image (0 or one unit vector e_i, since B e_i is row
// i of B and B (s ^ e_i) = q ^ B_i), or wt(de) <= 1 and de = m = 0 or e_i.  So
// one byte per syndrome -- idx (bits 0-3; 15: none), flag (bit 4: de = B (s ^
// e_idx), else de = e_idx) and the count n (bits 5-7: 0-3, 4 = uncorrectable,
// which keeps the data) -- plus linear pieces: spread(B (s ^ e_i)) =
// spread(B s) ^ spread(B_i) and spread(B s) from two 64-entry tables.
// Words: [0, 64) T0[i] = spread(i) | par(i) << 20, [64, 128) T1 for i << 6,
// [128, 192) U0[i] = spread(par(i)), [192, 256) U1 for i << 6, [256, 288)
// K[flag << 4 | idx] = spread(flag ? B_idx : e_idx) (0 past idx 11), then the
// 4096 class bytes.
constexpr int kBcBytes = 288;  // word offset of the class bytes
constexpr int kBcWords = kBcBytes + 1024;
constexpr int kBcAlloc = 1536;  // 6 KiB: whole 1 KiB LDS-DMA chunks (STAGE 2)

static void bc_tables(uint32_t *t) {
  auto sp = [](uint32_t d) { return golay_spread(d & 0xFFFu); };
  for (uint32_t i = 0; i < 64; ++i) {
    t[i] = sp(i) | golay_parity12(i) << 20;
    t[64 + i] = sp(i << 6) | golay_parity12(i << 6) << 20;
    t[128 + i] = sp(golay_parity12(i));
    t[192 + i] = sp(golay_parity12(i << 6));
  }
  for (uint32_t k = 0; k < 32; ++k) {
    const uint32_t idx = k & 15u, flag = k >> 4;
    t[256 + k] = idx < 12 ? sp(flag ? golay_parity12(1u << idx) : 1u << idx) : 0u;
  }
  uint8_t *c = reinterpret_cast<uint8_t *>(t + kBcBytes);
  for (int s = 0; s < 4096; ++s) c[s] = 0x80 | 0x0F;  // uncorrectable: n = 4, de = 0
  // coset leaders of weight <= 3 (unique: minimum distance 8)
  for (uint32_t e = 0; e < (1u << 24); ++e) {
    const int w = __builtin_popcount(e);
    if (w > 3) continue;
    const uint32_t de = e & 0xFFFu, pe = e >> 12;
    const uint32_t s = golay_parity12(de) ^ pe;
    uint32_t code = 0xFFu;
    for (uint32_t flag = 0; flag < 2 && code == 0xFFu; ++flag)
      for (uint32_t idx = 0; idx < 16 && code == 0xFFu; ++idx) {
        if (idx >= 12 && idx < 15) continue;
        const uint32_t m = idx < 12 ? 1u << idx : 0u;
        if ((flag ? golay_parity12(s ^ m) : m) == de) code = idx | flag << 4 | (uint32_t)w << 5;
      }
    c[s] = (uint8_t)code;
  }
}

// the tables on the device (built once; never freed: experiment processes)
static const uint32_t *bc_tables_dev() {
  static uint32_t *dev = nullptr;
  if (!dev) {
    std::vector<uint32_t> h(kBcAlloc, 0u);
    bc_tables(h.data());
    uint32_t *d = nullptr;
    if (hipMalloc(&d, sizeof(uint32_t) * h.size()) != hipSuccess ||
        hipMemcpy(d, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice) != hipSuccess)
      return nullptr;
    dev = d;
  }
  return dev;
}

// one codeword: spread nibbles (bytes 0-2) of the corrected data and the
// count n (0-3, 4 = uncorrectable, data kept), from the tables in LDS
__device__ __forceinline__ uint32_t bc_decode(const uint32_t *tab, uint32_t cw, uint32_t &n) {
  const uint8_t *c8 = reinterpret_cast<const uint8_t *>(tab + kBcBytes);
  const uint32_t p = tab[cw & 63u] ^ tab[64 + ((cw >> 6) & 63u)];
  const uint32_t s = ((cw >> 12) ^ (p >> 20)) & 0xFFFu;
  const uint32_t us = tab[128 + (s & 63u)] ^ tab[192 + (s >> 6)];
  const uint32_t b = c8[s];
  const uint32_t k = tab[256 + (b & 31u)];
  const uint32_t mask = (uint32_t)__builtin_amdgcn_sbfe((int)b, 4, 1);
  n = b >> 5;
  return __builtin_amdgcn_bitop3_b32(p, (mask & us) ^ k, 0x000F0F0Fu, 0x28);
}

}  // namespace exp
}  // namespace kvecc
