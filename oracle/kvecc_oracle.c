/*
 * kvecc_oracle.c -- plain-C restatement of the reference codec path.
 *
 * TEST INFRASTRUCTURE ONLY (see kvecc_oracle.h).  Written for obviousness, not
 * speed: bit-by-bit loops exactly as the reference Triton kernels state them.
 * Compile with -ffp-contract=off so float expressions round like the kernels.
 *
 * Parity: pinned against the tests/golden fixtures (generated from the reference
 * Triton kernels under TRITON_INTERPRET=1 by tools/gen_golden.py).
 */
#include "kvecc_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* Golay(24,12) code definition                                              */
/* ------------------------------------------------------------------------ */

/* The 12x12 B matrix, config.py:329-347 (row j lists the parity bits that data
 * bit j feeds).  Stored one row per word, bit i = B[j][i]. */
static const uint8_t GOLAY_B[12][12] = {
    {1, 1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 1}, {1, 0, 1, 1, 1, 0, 0, 0, 1, 0, 1, 1},
    {0, 1, 1, 1, 0, 0, 0, 1, 0, 1, 1, 1}, {1, 1, 1, 0, 0, 0, 1, 0, 1, 1, 0, 1},
    {1, 1, 0, 0, 0, 1, 0, 1, 1, 0, 1, 1}, {1, 0, 0, 0, 1, 0, 1, 1, 0, 1, 1, 1},
    {0, 0, 0, 1, 0, 1, 1, 0, 1, 1, 1, 1}, {0, 0, 1, 0, 1, 1, 0, 1, 1, 1, 0, 1},
    {0, 1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 1}, {1, 0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 1},
    {0, 1, 1, 0, 1, 1, 1, 0, 0, 0, 1, 1}, {1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0},
};

static int parity32(uint32_t x) {
  int p = 0;
  while (x) {
    p ^= (int)(x & 1u);
    x >>= 1;
  }
  return p;
}

static int popcount32(uint32_t x) {
  int c = 0;
  while (x) {
    c += (int)(x & 1u);
    x >>= 1;
  }
  return c;
}

/* column i of B as a 12-bit mask: bit j = B[j][i]  (golay_triton.py:59-70) */
static uint32_t golay_bcol(int i) {
  uint32_t m = 0;
  for (int j = 0; j < 12; ++j)
    if (GOLAY_B[j][i]) m |= 1u << j;
  return m;
}

void oracle_golay_h_row_masks(uint32_t out[12]) {
  /* H = [B^T | I12]: row i = column i of B in bits 0..11, plus bit 12+i. */
  for (int i = 0; i < 12; ++i) out[i] = golay_bcol(i) | (1u << (12 + i));
}

static uint32_t golay_syndrome(uint32_t word, const uint32_t h[12]) {
  uint32_t s = 0;
  for (int i = 0; i < 12; ++i) s |= (uint32_t)parity32(word & h[i]) << i;
  return s;
}

void oracle_golay_syndrome_table(int32_t out[4096]) {
  uint32_t h[12];
  oracle_golay_h_row_masks(h);
  for (int s = 0; s < 4096; ++s) out[s] = -1;
  out[0] = 0;
  /* weight 1: unconditional store (config.py:433-436) */
  for (int i = 0; i < 24; ++i) {
    uint32_t e = 1u << i;
    out[golay_syndrome(e, h)] = (int32_t)e;
  }
  /* weight 2 then 3, lexicographic, first pattern wins (config.py:438-453) */
  for (int i = 0; i < 24; ++i)
    for (int j = i + 1; j < 24; ++j) {
      uint32_t e = (1u << i) | (1u << j);
      uint32_t s = golay_syndrome(e, h);
      if (out[s] == -1) out[s] = (int32_t)e;
    }
  for (int i = 0; i < 24; ++i)
    for (int j = i + 1; j < 24; ++j)
      for (int k = j + 1; k < 24; ++k) {
        uint32_t e = (1u << i) | (1u << j) | (1u << k);
        uint32_t s = golay_syndrome(e, h);
        if (out[s] == -1) out[s] = (int32_t)e;
      }
}

/* ------------------------------------------------------------------------ */
/* Hamming(7,4) / (8,4)                                                      */
/* ------------------------------------------------------------------------ */

/* 3-bit syndrome -> bit position, -1 = none (config.py:131-161) */
static const int8_t HAMMING_LUT[8] = {-1, 4, 5, 0, 6, 1, 2, 3};

static uint8_t h74_word(uint8_t v) {
  int d0 = v & 1, d1 = (v >> 1) & 1, d2 = (v >> 2) & 1, d3 = (v >> 3) & 1;
  int p0 = d0 ^ d1 ^ d3, p1 = d0 ^ d2 ^ d3, p2 = d1 ^ d2 ^ d3;
  return (uint8_t)(d0 | d1 << 1 | d2 << 2 | d3 << 3 | p0 << 4 | p1 << 5 | p2 << 6);
}

static int h74_syndrome(uint8_t c) {
  int c0 = c & 1, c1 = (c >> 1) & 1, c2 = (c >> 2) & 1, c3 = (c >> 3) & 1;
  int c4 = (c >> 4) & 1, c5 = (c >> 5) & 1, c6 = (c >> 6) & 1;
  int s0 = c0 ^ c1 ^ c3 ^ c4;
  int s1 = c0 ^ c2 ^ c3 ^ c5;
  int s2 = c1 ^ c2 ^ c3 ^ c6;
  return s0 | s1 << 1 | s2 << 2;
}

void oracle_h74_encode(const uint8_t *in, uint8_t *out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) out[i] = h74_word(in[i]);
}

void oracle_h74_decode(const uint8_t *cw, uint8_t *data, uint8_t *flag, int64_t n,
                       int64_t *stats) {
  int64_t corrected = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint8_t c = cw[i];
    int s = h74_syndrome(c); /* bit 7 never enters the syndrome */
    int pos = HAMMING_LUT[s];
    uint8_t fix = pos >= 0 ? (uint8_t)(1u << pos) : 0;
    data[i] = (uint8_t)((c ^ fix) & 0x0F);
    flag[i] = (uint8_t)(s != 0);
    corrected += (s != 0);
  }
  if (stats) stats[0] = corrected;
}

void oracle_h84_encode(const uint8_t *in, uint8_t *out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    uint8_t h7 = h74_word(in[i]);
    out[i] = (uint8_t)(h7 | (parity32(h7) << 7));
  }
}

void oracle_h84_decode(const uint8_t *cw, uint8_t *data, uint8_t *etype, int64_t n,
                       int64_t *stats) {
  int64_t single = 0, dbl = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint8_t c = cw[i];
    uint8_t h7 = c & 0x7F;
    int stored = (c >> 7) & 1;
    int s = h74_syndrome(h7);
    int perr = stored != parity32(h7);
    int t = (s == 0) ? (perr ? 3 : 0) : (perr ? 1 : 2);
    int pos = HAMMING_LUT[s];
    uint8_t fix = (t == 1 && pos >= 0) ? (uint8_t)(1u << pos) : 0;
    data[i] = (uint8_t)((h7 ^ fix) & 0x0F); /* type 2 keeps data (:200-206) */
    etype[i] = (uint8_t)t;
    single += (t == 1);
    dbl += (t == 2);
  }
  if (stats) {
    stats[0] = single;
    stats[1] = dbl;
  }
}

/* ------------------------------------------------------------------------ */
/* Golay(24,12) encode / decode                                              */
/* ------------------------------------------------------------------------ */

void oracle_golay_encode(const uint8_t *trip, int32_t *cw, int64_t m) {
  uint32_t col[12];
  for (int i = 0; i < 12; ++i) col[i] = golay_bcol(i);
  for (int64_t k = 0; k < m; ++k) {
    uint32_t d = (uint32_t)(trip[3 * k] & 0xF) | (uint32_t)(trip[3 * k + 1] & 0xF) << 4 |
                 (uint32_t)(trip[3 * k + 2] & 0xF) << 8;
    uint32_t p = 0;
    for (int i = 0; i < 12; ++i) p |= (uint32_t)parity32(d & col[i]) << i;
    cw[k] = (int32_t)(d | p << 12);
  }
}

void oracle_golay_decode(const int32_t *cw, uint8_t *trip, uint8_t *count, int64_t m,
                         int64_t *stats) {
  static int32_t table[4096];
  static uint32_t h[12];
  static int ready = 0;
  if (!ready) {
    oracle_golay_syndrome_table(table);
    oracle_golay_h_row_masks(h);
    ready = 1;
  }
  int64_t bits = 0, unc = 0;
  for (int64_t k = 0; k < m; ++k) {
    uint32_t w = (uint32_t)cw[k];
    uint32_t s = golay_syndrome(w, h); /* masks are 24-bit: high byte ignored */
    int32_t e = table[s];
    int ok = e >= 0;
    uint32_t fixed = ok ? (w ^ (uint32_t)e) : w;
    uint32_t d = fixed & 0xFFF;
    trip[3 * k] = (uint8_t)(d & 0xF);
    trip[3 * k + 1] = (uint8_t)((d >> 4) & 0xF);
    trip[3 * k + 2] = (uint8_t)((d >> 8) & 0xF);
    int c = ok ? popcount32((uint32_t)e) : 4;
    count[k] = (uint8_t)c;
    if (c < 4)
      bits += c;
    else
      unc += 1;
  }
  if (stats) {
    stats[0] = bits;
    stats[1] = unc;
  }
}

/* ------------------------------------------------------------------------ */
/* Triton Philox4x32-10 and tl.rand                                          */
/* ------------------------------------------------------------------------ */

void oracle_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                          uint32_t k0, uint32_t k1, uint32_t out[4]) {
  for (int r = 0; r < 10; ++r) {
    uint32_t old0 = c0, old2 = c2;
    uint64_t prod_b = (uint64_t)0xCD9E8D57u * old2;
    uint64_t prod_a = (uint64_t)0xD2511F53u * old0;
    c0 = (uint32_t)(prod_b >> 32) ^ c1 ^ k0;
    c2 = (uint32_t)(prod_a >> 32) ^ c3 ^ k1;
    c1 = (uint32_t)prod_b;
    c3 = (uint32_t)prod_a;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

float oracle_uint_to_uniform(uint32_t x) {
  int32_t v = (int32_t)x;
  if (v < 0) v = ~v; /* -x-1 without signed overflow */
  volatile float f = (float)v;
  return f * 4.6566127342e-10f;
}

/* tl.rand(seed_i32, offset_i32): key = seed sign-extended to 64 bits,
 * counter = (offset, 0, 0, 0), first output word. */
static void tl_rand4(int32_t seed, int32_t offset, float u[4]) {
  uint64_t key = (uint64_t)(int64_t)seed;
  uint32_t o[4];
  oracle_philox4x32_10((uint32_t)offset, 0u, 0u, 0u, (uint32_t)key, (uint32_t)(key >> 32),
                       o);
  for (int i = 0; i < 4; ++i) u[i] = oracle_uint_to_uniform(o[i]);
}

static int32_t wrap32(int64_t v) { return (int32_t)(uint32_t)(uint64_t)v; }

/* per-bit kernels: base = seed*(N*n_bits) + off*n_bits, key of bit b = base + b
 * (all int32 arithmetic, fault_injection_triton.py:247,322) */
static uint32_t flip_mask_bits(int64_t seed, int64_t global_n, int64_t off, int n_bits,
                               int nb_eff, float ber) {
  uint64_t base = (uint64_t)seed * (uint64_t)(global_n * n_bits) + (uint64_t)off * (uint64_t)n_bits;
  uint32_t mask = 0;
  for (int b = 0; b < nb_eff; ++b) {
    float u[4];
    tl_rand4(wrap32((int64_t)(base + (uint64_t)b)), wrap32(off), u);
    if (u[0] < ber) mask |= 1u << b;
  }
  return mask;
}

void oracle_inject_u8(const uint8_t *in, uint8_t *out, uint8_t *count, int64_t n,
                      int n_bits, int64_t seed, float ber, int64_t global_n,
                      int64_t offset0, int64_t *stats) {
  /* bit 0 is always drawn; bits 1..7 when n_bits allows (:249-294) */
  int nb = n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits);
  int64_t flips = 0, affected = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t m = flip_mask_bits(seed, global_n, offset0 + i, n_bits, nb, ber);
    out[i] = (uint8_t)(in[i] ^ m);
    int c = popcount32(m);
    count[i] = (uint8_t)c;
    flips += c;
    affected += c > 0;
  }
  if (stats) {
    stats[0] = flips;
    stats[1] = affected;
  }
}

/* the shim's per-row injection (kv_cache/ecc_shim.py:594-603, 644-652): each of
 * `rows` contiguous rows of row_len codewords is injected as its own tensor,
 * row r with seed seed0 + r (the write loop's config.seed + _injection_count,
 * counted once per (batch, position, head) row) */
void oracle_inject_rows_u8(const uint8_t *in, uint8_t *out, int64_t rows, int64_t row_len,
                           int n_bits, int64_t seed0, float ber, int64_t *stats) {
  uint8_t *cnt = (uint8_t *)malloc(row_len > 0 ? (size_t)row_len : 1u);
  int64_t flips = 0, affected = 0, st[2];
  for (int64_t r = 0; r < rows; ++r) {
    oracle_inject_u8(in + r * row_len, out + r * row_len, cnt, row_len, n_bits, seed0 + r, ber,
                     row_len, 0, st);
    flips += st[0];
    affected += st[1];
  }
  free(cnt);
  if (stats) {
    stats[0] = flips;
    stats[1] = affected;
  }
}

void oracle_inject_i32(const int32_t *in, int32_t *out, uint8_t *count, int64_t n,
                       int n_bits, int64_t seed, float ber, int64_t global_n,
                       int64_t offset0, int64_t *stats) {
  int nb = n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits); /* :324-325 */
  int64_t flips = 0, affected = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t m = flip_mask_bits(seed, global_n, offset0 + i, n_bits, nb, ber);
    out[i] = (int32_t)((uint32_t)in[i] ^ m);
    int c = popcount32(m);
    count[i] = (uint8_t)c;
    flips += c;
    affected += c > 0;
  }
  if (stats) {
    stats[0] = flips;
    stats[1] = affected;
  }
}

/* rand4x variants: key of batch k = seed*N + off + k*N, outputs c0..c3 -> bits
 * 4k..4k+3 (:82-128, :161-219) */
static uint32_t flip_mask_vec(int64_t seed, int64_t n, int64_t off, int nb_eff, float ber) {
  uint32_t mask = 0;
  uint64_t base = (uint64_t)seed * (uint64_t)n + (uint64_t)off;
  for (int k = 0; 4 * k < nb_eff; ++k) {
    float u[4];
    tl_rand4(wrap32((int64_t)(base + (uint64_t)k * (uint64_t)n)), wrap32(off), u);
    for (int j = 0; j < 4 && 4 * k + j < nb_eff; ++j)
      if (u[j] < ber) mask |= 1u << (4 * k + j);
  }
  return mask;
}

void oracle_inject_u8_vectorized(const uint8_t *in, uint8_t *out, uint8_t *count,
                                 int64_t n, int n_bits, int64_t seed, float ber,
                                 int64_t *stats) {
  int nb = n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits); /* r0 always used */
  int64_t flips = 0, affected = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t m = flip_mask_vec(seed, n, i, nb, ber);
    out[i] = (uint8_t)(in[i] ^ m);
    int c = popcount32(m);
    count[i] = (uint8_t)c;
    flips += c;
    affected += c > 0;
  }
  if (stats) {
    stats[0] = flips;
    stats[1] = affected;
  }
}

void oracle_inject_i32_vectorized(const int32_t *in, int32_t *out, uint8_t *count,
                                  int64_t n, int n_bits, int64_t seed, float ber,
                                  int64_t *stats) {
  int nb = n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits);
  int64_t flips = 0, affected = 0;
  for (int64_t i = 0; i < n; ++i) {
    uint32_t m = nb > 0 ? flip_mask_vec(seed, n, i, nb, ber) : 0u;
    out[i] = (int32_t)((uint32_t)in[i] ^ m);
    int c = popcount32(m);
    count[i] = (uint8_t)c;
    flips += c;
    affected += c > 0;
  }
  if (stats) {
    stats[0] = flips;
    stats[1] = affected;
  }
}

/* ------------------------------------------------------------------------ */
/* Interpolation                                                             */
/* ------------------------------------------------------------------------ */

void oracle_interpolate(const uint8_t *q, const uint8_t *err, uint8_t *out,
                        int64_t outer, int64_t len, int64_t inner) {
  for (int64_t o = 0; o < outer; ++o)
    for (int64_t l = 0; l < len; ++l)
      for (int64_t c = 0; c < inner; ++c) {
        int64_t base = o * len * inner + c;
        int64_t i = base + l * inner;
        int64_t li = l > 0 ? l - 1 : 0;
        int64_t ri = l + 1 < len ? l + 1 : len - 1;
        float v = (float)q[i];
        float left = (float)q[base + li * inner];
        float right = (float)q[base + ri * inner];
        volatile float sum = left + right;
        float interp = sum * 0.5f;
        float r = err[i] == 2 ? interp : v;
        volatile float rh = r + 0.5f;
        float c15 = rh < 15.0f ? rh : 15.0f;
        float c0 = c15 > 0.0f ? c15 : 0.0f;
        out[i] = (uint8_t)c0;
      }
}

/* ------------------------------------------------------------------------ */
/* Quantization                                                              */
/* ------------------------------------------------------------------------ */

/* rule 0: scale = amax / 7 (IEEE), torch on CPU tensors; rule 1: amax * RN(1/7),
 * torch's tensor / Python scalar on a GPU (paged_cache_ecc.py:330). */
void oracle_quantize_rows(const float *x, int64_t rows, int64_t d, int rule, uint8_t *q,
                          float *scales) {
  const volatile float inv7 = 1.0f / 7.0f;
  for (int64_t r = 0; r < rows; ++r) {
    const float *row = x + r * d;
    float amax = 0.0f;
    for (int64_t j = 0; j < d; ++j) {
      float a = fabsf(row[j]);
      if (a > amax) amax = a;
    }
    volatile float scale = rule ? amax * inv7 : amax / 7.0f;
    if (scale == 0.0f) scale = 1.0f;
    scales[r] = scale;
    for (int64_t j = 0; j < d; ++j) {
      volatile float t = row[j] / scale;
      float v = rintf(t); /* default rounding mode: half to even */
      if (v > 7.0f) v = 7.0f;
      if (v < -8.0f) v = -8.0f;
      q[r * d + j] = (uint8_t)(int)(v + 8.0f);
    }
  }
}

void oracle_decode_dequant_h84(const uint8_t *cw, const float *scales, int64_t rows,
                               int64_t d, float *out, int64_t *corrected) {
  int64_t single = 0;
  for (int64_t r = 0; r < rows; ++r)
    for (int64_t j = 0; j < d; ++j) {
      uint8_t data, t;
      int64_t st[2];
      oracle_h84_decode(cw + r * d + j, &data, &t, 1, st);
      if (t == 2) data = 0; /* fused_kernels.py:344 */
      single += (t == 1);
      volatile float v = (float)data - 8.0f;
      out[r * d + j] = v * scales[r];
    }
  if (corrected) *corrected = single;
}
