// codec_math.h -- the codec algebra, shared by the gfx950 kernels and the
// host ("cpu" backend) implementation: one definition of every bit operation.
// The Hamming codecs have two forms of the same function -- v_perm byte tables
// on the device, shifts/XORs on the host -- which tests/native/codec_math_check.cpp
// proves equal on every byte value in every byte lane.
//
// References (ecc_codecs/triton_kernels/): hamming74_triton.py:48-162,
// hamming84_triton.py:50-209, golay_triton.py:99-295,
// fault_injection_triton.py:57-334 with triton/language/random.py:12-143,
// interpolation_triton.py:120-159, fused_kernels.py:18-357.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define KV_HD __host__ __device__ __forceinline__
#else
#define KV_HD inline
#endif

namespace kvecc {

// ---- bytes in a 32-bit word ----------------------------------------------------

// per-byte parity of four packed bytes: bit 0 of each byte = XOR of its 8 bits
KV_HD uint32_t byte_parity4(uint32_t y) {
  y ^= y >> 4;
  y ^= y >> 2;
  y ^= y >> 1;
  return y & 0x01010101u;
}

// a ^ b ^ c in one gfx950 v_bitop3_b32 (truth table 0x96); gfx9 has no v_xor3
KV_HD uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// ---- Hamming(7,4) / Hamming(8,4), four codewords per word (SWAR) -------------

// v_perm_b32 for selectors 0..7: byte i = byte sel.byte[i] of (hi:lo)
KV_HD uint32_t byte_perm(uint32_t hi, uint32_t lo, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(hi, lo, sel);
#else
  const uint64_t t = (uint64_t)hi << 32 | lo;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r |= (uint32_t)(t >> (8 * ((sel >> (8 * i)) & 7)) & 0xFFu) << (8 * i);
  return r;
#endif
}

// Encoders.  Parity is linear in the data bits: the device looks the parity
// byte of (d0,d1,d2) up in an 8-entry v_perm table and XORs in d3's (it flips
// p0, p1 and p2; the H84 overall parity P reduces to d0^d1^d2).
constexpr uint64_t h_enc_table(bool overall) {
  uint64_t t = 0;
  for (uint32_t v = 0; v < 8; ++v) {
    const uint32_t d0 = v & 1, d1 = v >> 1 & 1, d2 = v >> 2 & 1;
    const uint32_t e = (d0 ^ d1) << 4 | (d0 ^ d2) << 5 | (d1 ^ d2) << 6 |
                       (overall ? (d0 ^ d1 ^ d2) << 7 : 0u);
    t |= (uint64_t)e << (8 * v);
  }
  return t;
}
constexpr uint64_t kH74Enc = h_enc_table(false), kH84Enc = h_enc_table(true);

template <bool OVERALL>
KV_HD uint32_t h_encode4_tables(uint32_t w) {
  const uint32_t x = w & 0x0F0F0F0Fu;
  constexpr uint64_t t = OVERALL ? kH84Enc : kH74Enc;
  const uint32_t p012 = byte_perm((uint32_t)(t >> 32), (uint32_t)t, x & 0x07070707u);
  const uint32_t p3 = byte_perm(0u, 0x7000u, (x >> 3) & 0x01010101u);  // d3 -> 0x70
  return x | (p012 ^ p3);
}

template <bool OVERALL>
KV_HD uint32_t h_encode4_shifts(uint32_t w) {
  const uint32_t x = w & 0x0F0F0F0Fu;
  uint32_t d0 = x & 0x01010101u, d1 = (x >> 1) & 0x01010101u;
  uint32_t d2 = (x >> 2) & 0x01010101u, d3 = (x >> 3) & 0x01010101u;
  // parity of the 7-bit word reduces to d0^d1^d2 (p0^p1^p2 = d3)
  return x | (d0 ^ d1 ^ d3) << 4 | (d0 ^ d2 ^ d3) << 5 | (d1 ^ d2 ^ d3) << 6 |
         (OVERALL ? (d0 ^ d1 ^ d2) << 7 : 0u);
}

// the device uses the tables, the host the shift form (tests/native checks they agree)
template <bool OVERALL>
KV_HD uint32_t h_encode4(uint32_t w) {
#if defined(__HIP_DEVICE_COMPILE__)
  return h_encode4_tables<OVERALL>(w);
#else
  return h_encode4_shifts<OVERALL>(w);
#endif
}

KV_HD uint32_t h74_encode4(uint32_t w) { return h_encode4<false>(w); }
KV_HD uint32_t h84_encode4(uint32_t w) { return h_encode4<true>(w); }

// Syndrome bits (bit 0 of each byte) of four packed codewords, rows of H
// (config.py:296-304): s0 over bits {0,1,3,4}, s1 {0,2,3,5}, s2 {1,2,3,6}.
struct HammingSyndrome {
  uint32_t nz, fix;
  KV_HD explicit HammingSyndrome(uint32_t w) {
    uint32_t s0 = byte_parity4(w & 0x1B1B1B1Bu);
    uint32_t s1 = byte_parity4(w & 0x2D2D2D2Du);
    uint32_t s2 = byte_parity4(w & 0x4E4E4E4Eu);
    nz = s0 | s1 | s2;
    // data bit k is in error iff the syndrome equals column k of H:
    // d0 -> 3, d1 -> 5, d2 -> 6, d3 -> 7 (parity-bit positions 1,2,4 leave data alone)
    fix = (s0 & s1 & ~s2) | (s0 & ~s1 & s2) << 1 | (~s0 & s1 & s2) << 2 | (s0 & s1 & s2) << 3;
  }
};

// ---- the same syndromes through byte-permute tables (device) -----------------
//
// v_perm_b32 looks up four bytes at once in an 8-byte table held in two
// registers.  The syndrome is linear, so the bit fields {0,1,2}, {3,4,5} and
// {6,7} of each codeword byte index three tables whose entries are the XOR of
// the H columns of the set bits (d0 -> 3, d1 -> 5, d2 -> 6, d3 -> 7, p0 -> 1,
// p1 -> 2, p2 -> 4, P -> 0) in bits 0..2 and the field's parity replicated in
// bits 4..7; XORing the three lookups gives syndrome | overall-parity x 0xF.
// A fourth table maps the syndrome to the data-bit correction | nz << 4.
// About half the VALU work of the shift/XOR form; the host keeps that form.

// table entry for field value v whose bits carry H columns c0, c1, c2
constexpr uint32_t h_field_entry(uint32_t v, uint32_t c0, uint32_t c1, uint32_t c2) {
  return ((v & 1 ? c0 : 0) ^ (v & 2 ? c1 : 0) ^ (v & 4 ? c2 : 0)) |
         (((v ^ (v >> 1) ^ (v >> 2)) & 1) ? 0xF0u : 0u);
}
constexpr uint64_t h_field_table(uint32_t c0, uint32_t c1, uint32_t c2) {
  uint64_t t = 0;
  for (uint32_t v = 0; v < 8; ++v) t |= (uint64_t)h_field_entry(v, c0, c1, c2) << (8 * v);
  return t;
}
constexpr uint64_t kHField0 = h_field_table(3, 5, 6);  // d0 d1 d2
constexpr uint64_t kHField1 = h_field_table(7, 1, 2);  // d3 p0 p1
constexpr uint64_t kHField2 = h_field_table(4, 0, 0);  // p2 P (2-bit field)
// syndrome -> data correction (one-hot d0..d3 when the syndrome is a data
// column 3/5/6/7) | (syndrome != 0) << 4
constexpr uint64_t h_fix_table() {
  uint64_t t = 0;
  for (uint32_t s = 1; s < 8; ++s) {
    const uint32_t fix = s == 3 ? 1u : s == 5 ? 2u : s == 6 ? 4u : s == 7 ? 8u : 0u;
    t |= (uint64_t)(fix | 0x10u) << (8 * s);
  }
  return t;
}
constexpr uint64_t kHFix = h_fix_table();

// syndrome (bits 0..2) | overall parity x 0xF0 (bits 4..7), per byte
KV_HD uint32_t h_code4(uint32_t w) {
  const uint32_t a = byte_perm((uint32_t)(kHField0 >> 32), (uint32_t)kHField0, w & 0x07070707u);
  const uint32_t b = byte_perm((uint32_t)(kHField1 >> 32), (uint32_t)kHField1, (w >> 3) & 0x07070707u);
  const uint32_t c = byte_perm((uint32_t)(kHField2 >> 32), (uint32_t)kHField2, (w >> 6) & 0x03030303u);
  return a ^ b ^ c;
}

// Table form of the syndrome of four codewords: fx = correction (bits 0..3) |
// nz << 4 per byte; pe_rep = parity error replicated in bits 0..3 of each byte
// (bits 4..7 carry the next byte's syndrome: mask before use).
struct HammingTables {
  uint32_t fx, pe_rep;
  KV_HD explicit HammingTables(uint32_t w) {
    const uint32_t code = h_code4(w);
    fx = byte_perm((uint32_t)(kHFix >> 32), (uint32_t)kHFix, code & 0x07070707u);
    pe_rep = code >> 4;
  }
  KV_HD uint32_t nz() const { return (fx >> 4) & 0x01010101u; }
  KV_HD uint32_t pe() const { return pe_rep & 0x01010101u; }
};

// SECDED decode of four packed codewords: data nibbles, ErrorType bytes
KV_HD void h84_decode4(uint32_t w, uint32_t &data, uint32_t &type, uint32_t &n_single,
                       uint32_t &n_double) {
#if defined(__HIP_DEVICE_COMPILE__)
  const HammingTables t(w);
  data = (w ^ (t.fx & t.pe_rep)) & 0x0F0F0F0Fu;  // correct only SINGLE (pe && nz)
  const uint32_t pe = t.pe(), nz = t.nz();
#else
  HammingSyndrome s(w);
  const uint32_t pe = byte_parity4(w);  // stored overall parity != parity(bits 0..6)
  data = (w ^ (s.fix & (pe * 0x0Fu))) & 0x0F0F0F0Fu;  // correct only SINGLE (pe && nz)
  const uint32_t nz = s.nz;
#endif
  // (nz,pe) = (0,0)->0, (1,1)->1, (1,0)->2, (0,1)->3 (hamming84_triton.py:185-187)
  type = pe | (pe ^ nz) << 1;
  n_single += __builtin_popcount(pe & nz);
  n_double += __builtin_popcount(~pe & nz);
}

KV_HD void h74_decode4(uint32_t w, uint32_t &data, uint32_t &flag, uint32_t &n_flag) {
#if defined(__HIP_DEVICE_COMPILE__)
  const HammingTables t(w);  // bit 7 only moves the parity lane, unused here
  data = (w ^ t.fx) & 0x0F0F0F0Fu;  // doubles are miscorrected, as in the reference
  flag = t.nz();
#else
  HammingSyndrome s(w);
  data = (w ^ s.fix) & 0x0F0F0F0Fu;  // doubles are miscorrected, as in the reference
  flag = s.nz;
#endif
  n_flag += __builtin_popcount(flag);
}

// single nibble -> codeword (codec: 0 raw, 1 H74, 2 H84 -- KVECC_CODEC_*)
KV_HD uint32_t encode_nibble(uint32_t v, int codec) {
  if (codec == 2) return h84_encode4(v) & 0xFFu;
  if (codec == 1) return h74_encode4(v) & 0xFFu;
  return v;
}

// ---- INT4 row quantization (shim torch path, ecc_shim.py:572-580) -----------------

// correctly rounded fp32 division on both sides (torch's x / scale)
KV_HD float div_rn(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __fdiv_rn(a, b);
#else
  return a / b;
#endif
}

// scale = absmax / 7, 0 -> 1 (compute_quantization_scales, paged_cache_ecc.py:302-334).
// rule 0 (KVECC_SCALE_DIV7): IEEE division, torch on CPU tensors; rule 1
// (KVECC_SCALE_MUL_INV7): absmax * RN(1/7), torch's tensor / Python scalar on a GPU.
KV_HD float row_scale(float amax, int rule) {
  float s = rule ? amax * (1.0f / 7.0f) : div_rn(amax, 7.0f);
  return s == 0.0f ? 1.0f : s;
}

// rounded quotient clamped to [-8, 7], + 8
KV_HD uint32_t nibble_of_quotient(float quot) {
  float q = fminf(fmaxf(rintf(quot), -8.0f), 7.0f);
  return (uint32_t)(int)(q + 8.0f);
}

// round_half_even(x / scale) clamped to [-8, 7], + 8
KV_HD uint32_t quantize_nibble(float x, float scale) { return nibble_of_quotient(div_rn(x, scale)); }

// x / scale through a per-row reciprocal (Markstein): with inv = RN(1/scale),
// q0 = RN(x * inv) is within an ulp of x / scale, r = x - scale * q0 is exact
// under FMA, and RN(q0 + r * inv) is the correctly rounded quotient while no
// intermediate leaves the normal range.  Three ops instead of IEEE division's
// ~10.  The kernels take this path only for fp16/bf16 rows whose scale passes
// recip_ok; tests/test_quant_exhaustive.py checks it against IEEE division for
// every finite (value, row max) pair of both dtypes.
KV_HD bool recip_ok(float scale) { return scale >= 0x1p-64f && scale <= 0x1p64f; }
KV_HD float div_recip(float x, float scale, float inv) {
  const float q0 = x * inv;
  const float r = fmaf(-scale, q0, x);
  return fmaf(r, inv, q0);
}

// ---- Golay(24,12) ---------------------------------------------------------------

KV_HD uint32_t golay_pack(uint32_t b0, uint32_t b1, uint32_t b2) {
  return (b0 & 0xFu) | (b1 & 0xFu) << 4 | (b2 & 0xFu) << 8;
}

// 12 parity bits of a data word: bit i = parity(d & B_COL[i]) (golay_triton.py:59-70,130-155)
KV_HD uint32_t golay_parity12(uint32_t d) {
  constexpr uint32_t kBCol[12] = {0xA3B, 0xD1D, 0xE8E, 0xB47, 0xDA3, 0xED1,
                                  0xF68, 0xBB4, 0x9DA, 0x8ED, 0xC76, 0x7FF};
  uint32_t p = 0;
#pragma unroll
  for (int i = 0; i < 12; ++i) p |= ((uint32_t)__builtin_popcount(d & kBCol[i]) & 1u) << i;
  return p;
}

// 12-bit data word -> its three nibbles in three consecutive bytes
KV_HD uint32_t golay_spread(uint32_t d) {
  return (d & 0xFu) | (d & 0xF0u) << 4 | (d & 0xF00u) << 8;
}

// 4 consecutive triplets (12 bytes, little endian in 3 words) -> 4 data words
KV_HD void golay_unpack4(uint32_t w0, uint32_t w1, uint32_t w2, uint32_t d[4]) {
  d[0] = golay_pack(w0, w0 >> 8, w0 >> 16);
  d[1] = golay_pack(w0 >> 24, w1, w1 >> 8);
  d[2] = golay_pack(w1 >> 16, w1 >> 24, w2);
  d[3] = golay_pack(w2 >> 8, w2 >> 16, w2 >> 24);
}

// decode one codeword with the parity / correction tables (runtime.hip):
// returns the 12-bit data, `c` = corrected bits 0..3 or 4 (uncorrectable)
KV_HD uint32_t golay_decode1(uint32_t w, const uint16_t *par, const uint16_t *cor, uint32_t &c) {
  uint32_t lo = w & 0xFFFu;
  uint32_t e = cor[((w >> 12) & 0xFFFu) ^ par[lo]];
  c = e >> 12;
  return lo ^ (e & 0xFFFu);
}

// ---- Philox4x32-10 and the injection draw ------------------------------------

constexpr uint32_t kPhiloxA = 0xD2511F53u, kPhiloxB = 0xCD9E8D57u;
constexpr uint32_t kKeyA = 0x9E3779B9u, kKeyB = 0xBB67AE85u;

KV_HD uint32_t mulhi32(uint32_t a, uint32_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umulhi(a, b);  // v_mul_hi_u32 (the 64-bit mad form measured 1.6x slower)
#else
  return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}

KV_HD void philox_rounds(uint32_t &c0, uint32_t &c1, uint32_t &c2, uint32_t &c3, uint32_t k0,
                         uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hb = mulhi32(kPhiloxB, c2), lb = kPhiloxB * c2;
    uint32_t ha = mulhi32(kPhiloxA, c0), la = kPhiloxA * c0;
    c0 = xor3(hb, c1, k0);
    c2 = xor3(ha, c3, k1);
    c1 = lb;
    c3 = la;
    k0 += kKeyA;
    k1 += kKeyB;
  }
}

// tl.rand(key, ctr): first Philox output word for counter (ctr,0,0,0), key
// sign-extended to 64 bits (random.py:46-110)
KV_HD uint32_t philox_word0_k(uint32_t ctr, uint32_t k0, uint32_t k1) {
  uint32_t c0 = ctr, c1 = 0, c2 = 0, c3 = 0;
  philox_rounds(c0, c1, c2, c3, k0, k1);
  return c0;
}

KV_HD uint32_t philox_word0(uint32_t ctr, uint32_t key) {
  return philox_word0_k(ctr, key, (uint32_t)((int32_t)key >> 31));
}

// `uint_to_uniform_float(x) < ber` as an integer test against kvecc_ber_threshold
KV_HD bool philox_below(uint32_t x, uint32_t thr) {
  uint32_t f = x ^ (uint32_t)((int32_t)x >> 31);  // fold: x < 0 ? -x-1 : x
  return f < thr;
}

// The same test as one add and one compare: fold(x) < thr <=> x in [0, thr) or
// x in [2^32 - thr, 2^32) <=> (x + thr) mod 2^32 < 2 thr, valid for thr < 2^31.
// thr == 2^31 (ber >= ~1: every draw is below) is handled by the caller.
KV_HD uint32_t philox_below2(uint32_t x, uint32_t thr, uint32_t thr2) {
  return (uint32_t)(x + thr < thr2);
}

// flip mask of one element for the per-bit scheme; key_base = key of bit 0.
// The bits' keys are consecutive, so their sign-extension words k1 agree unless
// the run crosses 2^31 or 2^32; then k1 and its round offsets are shared
// across the bits (one add per round per element instead of per bit).
template <int NB>
KV_HD uint32_t philox_flip_mask(uint32_t key_base, uint32_t ctr, uint32_t thr, int nb_rt) {
  const int nb = NB >= 0 ? NB : nb_rt;
  if (nb <= 0) return 0;
  if (thr > 0x7FFFFFFFu) return nb >= 32 ? ~0u : (1u << nb) - 1;
  const uint32_t thr2 = 2 * thr;
  const uint32_t k1 = (uint32_t)((int32_t)key_base >> 31);
  const bool same_sign = k1 == (uint32_t)((int32_t)(key_base + (uint32_t)(nb - 1)) >> 31);
  uint32_t m = 0;
  if constexpr (NB >= 0) {
    if (same_sign) {
#pragma unroll
      for (int b = NB - 1; b >= 0; --b)
        m = m << 1 | philox_below2(philox_word0_k(ctr, key_base + b, k1), thr, thr2);
    } else {
#pragma unroll
      for (int b = NB - 1; b >= 0; --b)
        m = m << 1 | philox_below2(philox_word0(ctr, key_base + b), thr, thr2);
    }
  } else {
    for (int b = nb - 1; b >= 0; --b)
      m = m << 1 | philox_below2(philox_word0(ctr, key_base + b), thr, thr2);
  }
  return m;
}

// rand4x variant: batch k of 4 bits uses key seed*N + off + k*N, words c0..c3
KV_HD uint32_t philox_flip_mask_vec(uint32_t seedn, uint32_t nn, uint32_t off, uint32_t thr,
                                    int nb) {
  uint32_t m = 0;
  for (int k = 0; 4 * k < nb; ++k) {
    const uint32_t key = seedn + off + (uint32_t)k * nn;
    uint32_t c0 = off, c1 = 0, c2 = 0, c3 = 0;
    philox_rounds(c0, c1, c2, c3, key, (uint32_t)((int32_t)key >> 31));
    const uint32_t w[4] = {c0, c1, c2, c3};
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (4 * k + j < nb) m |= (uint32_t)philox_below(w[j], thr) << (4 * k + j);
  }
  return m;
}

// ---- interpolation, four bytes per word --------------------------------------------

// per byte: min(15, x)
KV_HD uint32_t sat15(uint32_t x) {
  uint32_t hi = (x >> 4) & 0x0F0F0F0Fu;                     // high nibble per byte
  uint32_t over = ((hi + 0x0F0F0F0Fu) >> 4) & 0x01010101u;  // 1 where x > 15
  return (x & ~(over * 0xFFu)) | (over * 0x0Fu);
}

// per byte: (a + b + 1) >> 1 without overflow
KV_HD uint32_t avg_up(uint32_t a, uint32_t b) { return (a | b) - (((a ^ b) >> 1) & 0x7F7F7F7Fu); }

// per byte: 0xFF where err == 2, else 0
KV_HD uint32_t is_double(uint32_t e) {
  uint32_t v = e ^ 0x02020202u;
  uint32_t nonzero = (((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
  return ((~nonzero & 0x80808080u) >> 7) * 0xFFu;
}

// err == 2 ? min(15, (L+R+1)>>1) : min(15, q)  -- the kernel's fp32 formula, exact
KV_HD uint32_t interp_word(uint32_t q, uint32_t l, uint32_t r, uint32_t e) {
  uint32_t m = is_double(e);
  return sat15((avg_up(l, r) & m) | (q & ~m));
}

}  // namespace kvecc
