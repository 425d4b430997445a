// cpu.hip -- the host ("cpu") codec backend: same algebra as the gfx950
// kernels (codec_math.h), run over host memory with std::thread workers.
//
// This is the explicit `backend="cpu"` of kvecc.backends (BASELINE config 1:
// Hamming(7,4) on the host, no GPU) -- never a fallback of the "hip" backend.
// Statistics are plain host uint64 arrays (+=), not the sharded device buffer.
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "kvecc_internal.h"

namespace kvecc {
namespace {

int clamp_threads(int threads, int64_t work, int64_t grain) {
  int hw = (int)std::thread::hardware_concurrency();
  if (threads <= 0) threads = hw > 0 ? hw : 1;
  int64_t useful = std::max<int64_t>(1, work / std::max<int64_t>(1, grain));
  return (int)std::max<int64_t>(1, std::min<int64_t>(threads, useful));
}

// run fn(begin, end, thread_index) over [0, n) in `threads` contiguous chunks
// whose boundaries are multiples of `align`
template <class F>
void parallel_for(int64_t n, int threads, int64_t align, F fn) {
  int t = clamp_threads(threads, n, 1 << 16);
  if (t == 1) {
    fn((int64_t)0, n, 0);
    return;
  }
  int64_t chunk = (n + t - 1) / t;
  chunk = (chunk + align - 1) / align * align;
  std::vector<std::thread> pool;
  for (int i = 0; i < t; ++i) {
    int64_t b = i * chunk, e = std::min<int64_t>(n, b + chunk);
    if (b >= e) break;
    pool.emplace_back(fn, b, e, i);
  }
  for (auto &th : pool) th.join();
}

inline uint32_t load4(const uint8_t *p) {
  uint32_t w;
  std::memcpy(&w, p, 4);
  return w;
}
inline void store4(uint8_t *p, uint32_t w) { std::memcpy(p, &w, 4); }

template <class Op>
void map_bytes(const uint8_t *in, uint8_t *out, int64_t n, int threads, Op op) {
  parallel_for(n, threads, 64, [&](int64_t b, int64_t e, int) {
    int64_t i = b;
    for (; i + 4 <= e; i += 4) store4(out + i, op(load4(in + i)));
    for (; i < e; ++i) out[i] = (uint8_t)op(in[i]);
  });
}

struct Acc2 {
  uint64_t a = 0, b = 0;
  char pad[48];
};

void add_stats(uint64_t *stats, const std::vector<Acc2> &acc, int n) {
  if (!stats) return;
  for (auto &x : acc) {
    stats[0] += x.a;
    if (n > 1) stats[1] += x.b;
  }
}

float load_x(const void *x, int dtype, int64_t i) {
  if (dtype == KVECC_F16) return __half2float(reinterpret_cast<const __half *>(x)[i]);
  if (dtype == KVECC_BF16) return __bfloat162float(reinterpret_cast<const __hip_bfloat16 *>(x)[i]);
  return reinterpret_cast<const float *>(x)[i];
}

void store_y(void *y, int dtype, int64_t i, float v) {
  if (dtype == KVECC_F16)
    reinterpret_cast<__half *>(y)[i] = __float2half_rn(v);
  else if (dtype == KVECC_BF16)
    reinterpret_cast<__hip_bfloat16 *>(y)[i] = __float2bfloat16(v);
  else
    reinterpret_cast<float *>(y)[i] = v;
}

bool bad(int64_t n) { return n < 0; }

}  // namespace
}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_cpu_hamming74_encode(const uint8_t *in, uint8_t *out, int64_t n, int threads) {
  if (bad(n)) return set_error(KVECC_EINVAL, "cpu_hamming74_encode: negative n");
  if (n && (!in || !out)) return set_error(KVECC_EINVAL, "cpu_hamming74_encode: null pointer");
  map_bytes(in, out, n, threads, [](uint32_t w) { return h74_encode4(w); });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_hamming84_encode(const uint8_t *in, uint8_t *out, int64_t n, int threads) {
  if (bad(n)) return set_error(KVECC_EINVAL, "cpu_hamming84_encode: negative n");
  if (n && (!in || !out)) return set_error(KVECC_EINVAL, "cpu_hamming84_encode: null pointer");
  map_bytes(in, out, n, threads, [](uint32_t w) { return h84_encode4(w); });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_hamming74_decode(const uint8_t *cw, uint8_t *data, uint8_t *flag, int64_t n,
                                         uint64_t *stats, int threads) {
  if (bad(n)) return set_error(KVECC_EINVAL, "cpu_hamming74_decode: negative n");
  if (n && (!cw || !data)) return set_error(KVECC_EINVAL, "cpu_hamming74_decode: null pointer");
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, n, 1 << 16)));
  parallel_for(n, threads, 64, [&](int64_t b, int64_t e, int t) {
    uint32_t c = 0;
    int64_t i = b;
    for (; i + 4 <= e; i += 4) {
      uint32_t d, f;
      h74_decode4(load4(cw + i), d, f, c);
      store4(data + i, d);
      if (flag) store4(flag + i, f);
    }
    for (; i < e; ++i) {
      uint32_t d, f;
      h74_decode4(cw[i], d, f, c);
      data[i] = (uint8_t)d;
      if (flag) flag[i] = (uint8_t)f;
    }
    acc[t].a += c;
  });
  add_stats(stats, acc, 1);
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_hamming84_decode(const uint8_t *cw, uint8_t *data, uint8_t *etype, int64_t n,
                                         uint64_t *stats, int threads) {
  if (bad(n)) return set_error(KVECC_EINVAL, "cpu_hamming84_decode: negative n");
  if (n && (!cw || !data)) return set_error(KVECC_EINVAL, "cpu_hamming84_decode: null pointer");
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, n, 1 << 16)));
  parallel_for(n, threads, 64, [&](int64_t b, int64_t e, int t) {
    uint32_t c1 = 0, c2 = 0;
    int64_t i = b;
    for (; i + 4 <= e; i += 4) {
      uint32_t d, ty;
      h84_decode4(load4(cw + i), d, ty, c1, c2);
      store4(data + i, d);
      if (etype) store4(etype + i, ty);
    }
    for (; i < e; ++i) {
      uint32_t d, ty;
      h84_decode4(cw[i], d, ty, c1, c2);
      data[i] = (uint8_t)d;
      if (etype) etype[i] = (uint8_t)ty;
    }
    acc[t].a += c1;
    acc[t].b += c2;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_golay_encode(const uint8_t *trip, int32_t *cw, int64_t m, int threads) {
  if (bad(m)) return set_error(KVECC_EINVAL, "cpu_golay_encode: negative m");
  if (m && (!trip || !cw)) return set_error(KVECC_EINVAL, "cpu_golay_encode: null pointer");
  static uint16_t par[4096];
  static bool ready = [] { build_golay_parity_table(par); return true; }();
  (void)ready;
  parallel_for(m, threads, 64, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      uint32_t d = golay_pack(trip[3 * i], trip[3 * i + 1], trip[3 * i + 2]);
      cw[i] = (int32_t)(d | (uint32_t)par[d] << 12);
    }
  });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_golay_decode(const int32_t *cw, uint8_t *trip, uint8_t *counts, int64_t m,
                                     uint64_t *stats, int threads) {
  if (bad(m)) return set_error(KVECC_EINVAL, "cpu_golay_decode: negative m");
  if (m && (!trip || !cw)) return set_error(KVECC_EINVAL, "cpu_golay_decode: null pointer");
  static uint16_t tab[8192];
  static bool ready = [] {
    build_golay_parity_table(tab);
    build_golay_correct_table(tab + 4096);
    return true;
  }();
  (void)ready;
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, m, 1 << 16)));
  parallel_for(m, threads, 64, [&](int64_t b, int64_t e, int t) {
    uint64_t bits = 0, unc = 0;
    for (int64_t i = b; i < e; ++i) {
      uint32_t c;
      uint32_t d = golay_decode1((uint32_t)cw[i], tab, tab + 4096, c);
      trip[3 * i] = (uint8_t)(d & 0xF);
      trip[3 * i + 1] = (uint8_t)(d >> 4 & 0xF);
      trip[3 * i + 2] = (uint8_t)(d >> 8);
      if (counts) counts[i] = (uint8_t)c;
      bits += c & 3u;
      unc += c >> 2;
    }
    acc[t].a += bits;
    acc[t].b += unc;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_golay_encode_rows(const uint8_t *nibbles, int32_t *cw, int64_t rows,
                                          int64_t d, int threads) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "cpu_golay_encode_rows: negative size");
  if (rows && d && (!nibbles || !cw)) return set_error(KVECC_EINVAL, "cpu_golay_encode_rows: null pointer");
  static uint16_t par[4096];
  static bool ready = [] { build_golay_parity_table(par); return true; }();
  (void)ready;
  const int64_t g = (d + 2) / 3;
  parallel_for(rows, threads, 1, [&](int64_t b, int64_t e, int) {
    for (int64_t r = b; r < e; ++r)
      for (int64_t k = 0; k < g; ++k) {
        const uint8_t *x = nibbles + r * d + 3 * k;
        const int64_t left = d - 3 * k;  // zero padding of the last group
        uint32_t dw = golay_pack(x[0], left > 1 ? x[1] : 0, left > 2 ? x[2] : 0);
        cw[r * g + k] = (int32_t)(dw | (uint32_t)par[dw] << 12);
      }
  });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_golay_decode_rows(const int32_t *cw, uint8_t *nibbles, int64_t rows,
                                          int64_t d, uint64_t *stats, int threads) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "cpu_golay_decode_rows: negative size");
  if (rows && d && (!nibbles || !cw)) return set_error(KVECC_EINVAL, "cpu_golay_decode_rows: null pointer");
  static uint16_t tab[8192];
  static bool ready = [] {
    build_golay_parity_table(tab);
    build_golay_correct_table(tab + 4096);
    return true;
  }();
  (void)ready;
  const int64_t g = (d + 2) / 3;
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, rows, 1)));
  parallel_for(rows, threads, 1, [&](int64_t b, int64_t e, int t) {
    uint64_t bits = 0, unc = 0;
    for (int64_t r = b; r < e; ++r)
      for (int64_t k = 0; k < g; ++k) {
        uint32_t c;
        const uint32_t dw = golay_decode1((uint32_t)cw[r * g + k], tab, tab + 4096, c);
        bits += c & 3u;
        unc += c >> 2;
        uint8_t *o = nibbles + r * d + 3 * k;
        const int64_t left = d - 3 * k;
        o[0] = (uint8_t)(dw & 0xF);
        if (left > 1) o[1] = (uint8_t)(dw >> 4 & 0xF);
        if (left > 2) o[2] = (uint8_t)(dw >> 8);
      }
    acc[t].a += bits;
    acc[t].b += unc;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

// packed Golay storage (host twins of packed.hip): one group of 8 codewords
// (12 nibble bytes, 24 codeword bytes, 1 flag byte) per work item
KVECC_API int kvecc_cpu_golay_encode_packed(const uint8_t *nibbles, uint8_t *codewords, int64_t m,
                                            int threads) {
  if (m < 0) return set_error(KVECC_EINVAL, "cpu_golay_encode_packed: negative m");
  if (m && (!nibbles || !codewords)) return set_error(KVECC_EINVAL, "cpu_golay_encode_packed: null pointer");
  static uint16_t par[4096];
  static bool ready = [] { build_golay_parity_table(par); return true; }();
  (void)ready;
  parallel_for((m + 7) / 8, threads, 1, [&](int64_t b, int64_t e, int) {
    for (int64_t g = b; g < e; ++g)
      for (int64_t k = 8 * g; k < m && k < 8 * g + 8; ++k) {
        uint32_t d = 0;
        for (int u = 0; u < 3; ++u) {
          const int64_t j = 3 * k + u;
          d |= (uint32_t)(nibbles[j >> 1] >> (4 * (j & 1)) & 0xF) << (4 * u);
        }
        const uint32_t c = d | (uint32_t)par[d] << 12;
        codewords[3 * k] = (uint8_t)c;
        codewords[3 * k + 1] = (uint8_t)(c >> 8);
        codewords[3 * k + 2] = (uint8_t)(c >> 16);
      }
  });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_golay_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                            uint8_t *uncorrectable, int64_t m, uint64_t *stats,
                                            int threads) {
  if (m < 0) return set_error(KVECC_EINVAL, "cpu_golay_decode_packed: negative m");
  if (m && (!nibbles || !codewords)) return set_error(KVECC_EINVAL, "cpu_golay_decode_packed: null pointer");
  static uint16_t tab[8192];
  static bool ready = [] {
    build_golay_parity_table(tab);
    build_golay_correct_table(tab + 4096);
    return true;
  }();
  (void)ready;
  const int64_t groups = (m + 7) / 8;
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, groups, 1 << 10)));
  parallel_for(groups, threads, 1, [&](int64_t b, int64_t e, int t) {
    uint64_t bits = 0, unc = 0;
    for (int64_t g = b; g < e; ++g) {
      uint32_t fl = 0;
      for (int64_t k = 8 * g; k < m && k < 8 * g + 8; ++k) {
        const uint32_t c = codewords[3 * k] | (uint32_t)codewords[3 * k + 1] << 8 |
                           (uint32_t)codewords[3 * k + 2] << 16;
        uint32_t cnt;
        const uint32_t d = golay_decode1(c, tab, tab + 4096, cnt);
        bits += cnt & 3u;
        unc += cnt >> 2;
        fl |= (cnt >> 2) << (k - 8 * g);
        for (int u = 0; u < 3; ++u) {
          const int64_t j = 3 * k + u;
          const uint32_t v = d >> (4 * u) & 0xFu;
          if ((j & 1) == 0)
            nibbles[j >> 1] = (uint8_t)v;  // high nibble: next value, or zero padding
          else
            nibbles[j >> 1] = (uint8_t)((nibbles[j >> 1] & 0x0Fu) | v << 4);
        }
      }
      if (uncorrectable) uncorrectable[g] = (uint8_t)fl;
    }
    acc[t].a += bits;
    acc[t].b += unc;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

// packed Hamming(8,4) (host twins of packed.hip): groups of 4 values share a
// type byte and two nibble bytes, one group per work item
KVECC_API int kvecc_cpu_hamming84_encode_packed(const uint8_t *nibbles, uint8_t *codewords,
                                                int64_t n, int threads) {
  if (n < 0) return set_error(KVECC_EINVAL, "cpu_hamming84_encode_packed: negative n");
  if (n && (!nibbles || !codewords)) return set_error(KVECC_EINVAL, "cpu_hamming84_encode_packed: null pointer");
  parallel_for(n, threads, 64, [&](int64_t b, int64_t e, int) {
    for (int64_t j = b; j < e; ++j)
      codewords[j] = (uint8_t)(h84_encode4(nibbles[j >> 1] >> (4 * (j & 1)) & 0xFu) & 0xFFu);
  });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_hamming84_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                                uint8_t *error_types, int64_t n, uint64_t *stats,
                                                int threads) {
  if (n < 0) return set_error(KVECC_EINVAL, "cpu_hamming84_decode_packed: negative n");
  if (n && (!nibbles || !codewords)) return set_error(KVECC_EINVAL, "cpu_hamming84_decode_packed: null pointer");
  const int64_t groups = (n + 3) / 4;
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, groups, 1 << 14)));
  parallel_for(groups, threads, 16, [&](int64_t b, int64_t e, int t) {
    uint32_t n1 = 0, n2 = 0;
    for (int64_t g = b; g < e; ++g) {
      uint32_t tb = 0;
      for (int64_t j = 4 * g; j < n && j < 4 * g + 4; ++j) {
        uint32_t d, ty;
        h84_decode4(codewords[j], d, ty, n1, n2);
        if ((j & 1) == 0)
          nibbles[j >> 1] = (uint8_t)d;  // high nibble: next value, or zero padding
        else
          nibbles[j >> 1] = (uint8_t)((nibbles[j >> 1] & 0x0Fu) | d << 4);
        tb |= ty << (2 * (j & 3));
      }
      if (error_types) error_types[g] = (uint8_t)tb;
    }
    acc[t].a += n1;
    acc[t].b += n2;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

}  // extern "C"

template <typename T>
static int cpu_inject(const T *in, T *out, uint8_t *counts, int64_t n, int n_bits, int64_t seed,
                      float ber, int64_t global_n, int64_t offset0, uint64_t *stats, int threads,
                      const char *name) {
  if (n < 0 || global_n < 0 || offset0 < 0) return set_error(KVECC_EINVAL, "%s: negative size", name);
  if (n && (!in || !out)) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  if (offset0 + n > global_n) return set_error(KVECC_EINVAL, "%s: shard exceeds global_n", name);
  const uint32_t seedmul = (uint32_t)((uint64_t)seed * (uint64_t)(uint32_t)((uint64_t)global_n * (uint64_t)n_bits));
  const uint32_t thr = kvecc_ber_threshold(ber);
  const int nb = sizeof(T) == 1 ? (n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits))
                                : (n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits));
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, n, 1 << 12)));
  parallel_for(n, threads, 64, [&](int64_t b, int64_t e, int t) {
    uint64_t flips = 0, hit = 0;
    for (int64_t i = b; i < e; ++i) {
      const uint32_t g = (uint32_t)(offset0 + i);
      const uint32_t m = philox_flip_mask<-1>(seedmul + g * (uint32_t)n_bits, g, thr, nb);
      out[i] = (T)((uint32_t)in[i] ^ m);
      uint32_t c = __builtin_popcount(m);
      if (counts) counts[i] = (uint8_t)c;
      flips += c;
      hit += c != 0;
    }
    acc[t].a += flips;
    acc[t].b += hit;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

template <typename T>
static int cpu_inject_rows(const T *in, T *out, int64_t rows, int64_t row_len, int n_bits,
                           int64_t seed_base, float ber, uint64_t *stats, int threads,
                           const char *name) {
  if (rows < 0 || row_len < 0) return set_error(KVECC_EINVAL, "%s: negative size", name);
  const int64_t total = rows * row_len;
  if (total && (!in || !out)) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  const uint32_t rowmul = (uint32_t)((uint64_t)row_len * (uint64_t)n_bits);
  const uint32_t sb = (uint32_t)(uint64_t)seed_base;
  const uint32_t thr = kvecc_ber_threshold(ber);
  const int nb = sizeof(T) == 1 ? (n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits))
                                : (n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits));
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, total, 1 << 12)));
  parallel_for(total, threads, 64, [&](int64_t b, int64_t e, int t) {
    uint64_t flips = 0, hit = 0;
    for (int64_t i = b; i < e; ++i) {
      const int64_t r = i / row_len;
      const uint32_t j = (uint32_t)(i - r * row_len);
      const uint32_t m = philox_flip_mask<-1>((sb + (uint32_t)r) * rowmul + j * (uint32_t)n_bits,
                                              j, thr, nb);
      out[i] = (T)((uint32_t)in[i] ^ m);
      uint32_t c = __builtin_popcount(m);
      flips += c;
      hit += c != 0;
    }
    acc[t].a += flips;
    acc[t].b += hit;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

template <typename T>
static int cpu_inject_vec(const T *in, T *out, uint8_t *counts, int64_t n, int n_bits,
                          int64_t seed, float ber, uint64_t *stats, int threads, const char *name) {
  if (n < 0) return set_error(KVECC_EINVAL, "%s: negative n", name);
  if (n && (!in || !out)) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  const uint32_t seedn = (uint32_t)((uint64_t)seed * (uint64_t)n);
  const uint32_t thr = kvecc_ber_threshold(ber);
  const int nb = sizeof(T) == 1 ? (n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits))
                                : (n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits));
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, n, 1 << 12)));
  parallel_for(n, threads, 64, [&](int64_t b, int64_t e, int t) {
    uint64_t flips = 0, hit = 0;
    for (int64_t i = b; i < e; ++i) {
      const uint32_t m = philox_flip_mask_vec(seedn, (uint32_t)n, (uint32_t)i, thr, nb);
      out[i] = (T)((uint32_t)in[i] ^ m);
      uint32_t c = __builtin_popcount(m);
      if (counts) counts[i] = (uint8_t)c;
      flips += c;
      hit += c != 0;
    }
    acc[t].a += flips;
    acc[t].b += hit;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

extern "C" {

KVECC_API int kvecc_cpu_inject_u8(const uint8_t *in, uint8_t *out, uint8_t *counts, int64_t n,
                                  int n_bits, int64_t seed, float ber, int64_t global_n,
                                  int64_t offset0, uint64_t *stats, int threads) {
  return cpu_inject<uint8_t>(in, out, counts, n, n_bits, seed, ber, global_n, offset0, stats,
                             threads, "cpu_inject_u8");
}

KVECC_API int kvecc_cpu_inject_i32(const int32_t *in, int32_t *out, uint8_t *counts, int64_t n,
                                   int n_bits, int64_t seed, float ber, int64_t global_n,
                                   int64_t offset0, uint64_t *stats, int threads) {
  return cpu_inject<int32_t>(in, out, counts, n, n_bits, seed, ber, global_n, offset0, stats,
                             threads, "cpu_inject_i32");
}

KVECC_API int kvecc_cpu_inject_u8_vectorized(const uint8_t *in, uint8_t *out, uint8_t *counts,
                                             int64_t n, int n_bits, int64_t seed, float ber,
                                             uint64_t *stats, int threads) {
  return cpu_inject_vec<uint8_t>(in, out, counts, n, n_bits, seed, ber, stats, threads,
                                 "cpu_inject_u8_vectorized");
}

KVECC_API int kvecc_cpu_inject_i32_vectorized(const int32_t *in, int32_t *out, uint8_t *counts,
                                              int64_t n, int n_bits, int64_t seed, float ber,
                                              uint64_t *stats, int threads) {
  return cpu_inject_vec<int32_t>(in, out, counts, n, n_bits, seed, ber, stats, threads,
                                 "cpu_inject_i32_vectorized");
}

KVECC_API int kvecc_cpu_inject_rows_u8(const uint8_t *in, uint8_t *out, int64_t rows,
                                       int64_t row_len, int n_bits, int64_t seed_base, float ber,
                                       uint64_t *stats, int threads) {
  return cpu_inject_rows<uint8_t>(in, out, rows, row_len, n_bits, seed_base, ber, stats, threads,
                                  "cpu_inject_rows_u8");
}

KVECC_API int kvecc_cpu_inject_rows_i32(const int32_t *in, int32_t *out, int64_t rows,
                                        int64_t row_len, int n_bits, int64_t seed_base, float ber,
                                        uint64_t *stats, int threads) {
  return cpu_inject_rows<int32_t>(in, out, rows, row_len, n_bits, seed_base, ber, stats, threads,
                                  "cpu_inject_rows_i32");
}

KVECC_API int kvecc_cpu_count_ne_u8(const uint8_t *a, const uint8_t *b, int64_t n, uint64_t *stats,
                                    int threads) {
  if (n < 0) return set_error(KVECC_EINVAL, "cpu_count_ne_u8: negative n");
  if (n == 0) return KVECC_OK;
  if (!a || !b || !stats) return set_error(KVECC_EINVAL, "cpu_count_ne_u8: null pointer");
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, n, 1 << 16)));
  parallel_for(n, threads, 1 << 16, [&](int64_t lo, int64_t hi, int t) {
    uint64_t c = 0;
    for (int64_t i = lo; i < hi; ++i) c += a[i] != b[i];
    acc[t].a += c;
  });
  add_stats(stats, acc, 1);
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_interpolate(const uint8_t *q, const uint8_t *err, uint8_t *out,
                                    int64_t outer, int64_t len, int64_t inner, int threads) {
  if (outer < 0 || len < 0 || inner < 0) return set_error(KVECC_EINVAL, "cpu_interpolate: negative size");
  const int64_t total = outer * len * inner;
  if (total && (!q || !err || !out)) return set_error(KVECC_EINVAL, "cpu_interpolate: null pointer");
  parallel_for(total, threads, 64, [&](int64_t b, int64_t e, int) {
    for (int64_t i = b; i < e; ++i) {
      const int64_t l = (i / inner) % len;
      const int64_t row = i - l * inner;
      const uint32_t left = q[row + (l > 0 ? l - 1 : 0) * inner];
      const uint32_t right = q[row + (l + 1 < len ? l + 1 : len - 1) * inner];
      out[i] = (uint8_t)interp_word(q[i], left, right, err[i]);
    }
  });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_quantize_encode_rows(const void *x, int x_dtype, int codec,
                                             int scale_rule, uint8_t *cw, float *scales,
                                             int64_t rows, int64_t d, int threads) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "cpu_quantize_encode_rows: negative size");
  if (rows == 0) return KVECC_OK;
  if (d == 0) return set_error(KVECC_EINVAL, "cpu_quantize_encode_rows: empty rows");
  if (!x || !cw || !scales) return set_error(KVECC_EINVAL, "cpu_quantize_encode_rows: null pointer");
  if (x_dtype < KVECC_F32 || x_dtype > KVECC_BF16)
    return set_error(KVECC_EINVAL, "cpu_quantize_encode_rows: bad dtype %d", x_dtype);
  if (codec < KVECC_CODEC_NONE || codec > KVECC_CODEC_H84)
    return set_error(KVECC_EINVAL, "cpu_quantize_encode_rows: bad codec %d", codec);
  if (scale_rule != KVECC_SCALE_DIV7 && scale_rule != KVECC_SCALE_MUL_INV7)
    return set_error(KVECC_EINVAL, "cpu_quantize_encode_rows: bad scale rule %d", scale_rule);
  parallel_for(rows, threads, 1, [&](int64_t b, int64_t e, int) {
    for (int64_t r = b; r < e; ++r) {
      float amax = 0.0f;
      for (int64_t j = 0; j < d; ++j) amax = std::max(amax, std::fabs(load_x(x, x_dtype, r * d + j)));
      const float scale = row_scale(amax, scale_rule);
      scales[r] = scale;
      for (int64_t j = 0; j < d; ++j)
        cw[r * d + j] = (uint8_t)encode_nibble(quantize_nibble(load_x(x, x_dtype, r * d + j), scale), codec);
    }
  });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_decode_dequant_h84_rows(const uint8_t *cw, const float *scales, void *out,
                                                int out_dtype, int64_t rows, int64_t d,
                                                int zero_doubles, uint64_t *stats, int threads) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "cpu_decode_dequant_h84_rows: negative size");
  if (rows == 0 || d == 0) return KVECC_OK;
  if (!cw || !scales || !out) return set_error(KVECC_EINVAL, "cpu_decode_dequant_h84_rows: null pointer");
  if (out_dtype < KVECC_F32 || out_dtype > KVECC_BF16)
    return set_error(KVECC_EINVAL, "cpu_decode_dequant_h84_rows: bad dtype %d", out_dtype);
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, rows, 1)));
  parallel_for(rows, threads, 1, [&](int64_t b, int64_t e, int t) {
    uint32_t n1 = 0, n2 = 0;
    for (int64_t r = b; r < e; ++r)
      for (int64_t j = 0; j < d; ++j) {
        uint32_t data, type;
        h84_decode4(cw[r * d + j], data, type, n1, n2);
        if (zero_doubles && type == 2) data = 0;
        store_y(out, out_dtype, r * d + j, ((float)data - 8.0f) * scales[r]);
      }
    acc[t].a += n1;
    acc[t].b += n2;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

// ---- shim write / read (host twins of shim.hip) ------------------------------

KVECC_API int kvecc_cpu_shim_write(const void *k, const void *v, int x_dtype, int64_t batch,
                                   int64_t seq, int64_t hkv, int64_t d, int codec,
                                   int scale_rule, int n_bits, int inject, float ber,
                                   int64_t seed0, void *k_cache,
                                   void *v_cache, float *k_scales, float *v_scales,
                                   const int32_t *block_table, int64_t num_layers,
                                   int64_t block_size, int64_t layer, int threads) {
  if (batch < 0 || seq < 0 || hkv < 0 || d < 0) return set_error(KVECC_EINVAL, "cpu_shim_write: negative size");
  if (batch == 0 || seq == 0 || hkv == 0) return KVECC_OK;
  if (d < 1) return set_error(KVECC_EINVAL, "cpu_shim_write: empty rows");
  if (codec < KVECC_CODEC_NONE || codec > KVECC_CODEC_GOLAY_PACKED)
    return set_error(KVECC_EINVAL, "cpu_shim_write: bad codec %d", codec);
  if (scale_rule != KVECC_SCALE_DIV7 && scale_rule != KVECC_SCALE_MUL_INV7)
    return set_error(KVECC_EINVAL, "cpu_shim_write: bad scale rule %d", scale_rule);
  if (x_dtype < KVECC_F32 || x_dtype > KVECC_BF16)
    return set_error(KVECC_EINVAL, "cpu_shim_write: bad dtype %d", x_dtype);
  if (num_layers < 1 || block_size < 1 || layer < 0 || layer >= num_layers)
    return set_error(KVECC_EINVAL, "cpu_shim_write: bad cache geometry");
  if (!k || !v || !k_cache || !v_cache || !k_scales || !v_scales || !block_table)
    return set_error(KVECC_EINVAL, "cpu_shim_write: null pointer");
  const bool packed = codec == KVECC_CODEC_GOLAY_PACKED;
  const bool golay = codec == KVECC_CODEC_GOLAY || packed;
  const int64_t g = golay ? (d + 2) / 3 : d;
  const uint32_t rowmul = (uint32_t)((uint64_t)g * (uint64_t)n_bits);
  const uint32_t thr = kvecc_ber_threshold(ber);
  const bool inj = inject != 0 && ber > 0.0f;
  const int nb = golay ? (n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits))
                       : (n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits));
  const int64_t per_side = seq * hkv;
  parallel_for(2 * per_side, threads, 1, [&](int64_t b, int64_t e, int) {
    std::vector<uint8_t> nib(3 * g + 3);
    for (int64_t item = b; item < e; ++item) {
      const int side = (int)(item / per_side);
      const int64_t rr = item - side * per_side;
      const int64_t pos = rr / hkv, h = rr - pos * hkv;
      const int64_t r = (batch - 1) * per_side + rr;
      const uint32_t key0 = ((uint32_t)(uint64_t)seed0 + (uint32_t)r + (uint32_t)side) * rowmul;
      const int64_t slot =
          (((int64_t)block_table[pos / block_size] * num_layers + layer) * hkv + h) * block_size +
          pos % block_size;
      const void *x = side ? v : k;
      float amax = 0.0f;
      for (int64_t j = 0; j < d; ++j) amax = std::max(amax, std::fabs(load_x(x, x_dtype, r * d + j)));
      const float scale = row_scale(amax, scale_rule);
      (side ? v_scales : k_scales)[slot] = scale;
      if (!golay) {
        uint8_t *c = reinterpret_cast<uint8_t *>(side ? v_cache : k_cache) + slot * g;
        for (int64_t j = 0; j < d; ++j) {
          uint32_t cw = encode_nibble(quantize_nibble(load_x(x, x_dtype, r * d + j), scale), codec);
          if (inj) cw ^= philox_flip_mask<-1>(key0 + (uint32_t)j * (uint32_t)n_bits, (uint32_t)j, thr, nb);
          c[j] = (uint8_t)cw;
        }
      } else {
        std::fill(nib.begin(), nib.end(), 0);
        for (int64_t j = 0; j < d; ++j) nib[j] = (uint8_t)quantize_nibble(load_x(x, x_dtype, r * d + j), scale);
        void *cache = side ? v_cache : k_cache;
        for (int64_t q = 0; q < g; ++q) {
          const uint32_t dw = golay_pack(nib[3 * q], nib[3 * q + 1], nib[3 * q + 2]);
          uint32_t cw = dw | golay_parity12(dw) << 12;
          if (inj) cw ^= philox_flip_mask<-1>(key0 + (uint32_t)q * (uint32_t)n_bits, (uint32_t)q, thr, nb);
          if (packed) {
            uint8_t *c = reinterpret_cast<uint8_t *>(cache) + slot * KVECC_GOLAY_PACKED_ROW(g) + 3 * q;
            c[0] = (uint8_t)cw;
            c[1] = (uint8_t)(cw >> 8);
            c[2] = (uint8_t)(cw >> 16);
          } else {
            reinterpret_cast<int32_t *>(cache)[slot * g + q] = (int32_t)cw;
          }
        }
      }
    }
  });
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_shim_read(const void *k_cache, const void *v_cache, const float *k_scales,
                                  const float *v_scales, const int32_t *block_table, int64_t ctx,
                                  int64_t hkv, int64_t d, int64_t num_layers, int64_t block_size,
                                  int64_t layer, int codec, int interp, void *k_out, void *v_out,
                                  int out_dtype, uint64_t *stats, int threads) {
  if (ctx < 0 || hkv < 0 || d < 0) return set_error(KVECC_EINVAL, "cpu_shim_read: negative size");
  if (ctx == 0 || hkv == 0 || d == 0) return KVECC_OK;
  if (codec < KVECC_CODEC_NONE || codec > KVECC_CODEC_GOLAY_PACKED)
    return set_error(KVECC_EINVAL, "cpu_shim_read: bad codec %d", codec);
  if (interp && codec != KVECC_CODEC_H84)
    return set_error(KVECC_EINVAL, "cpu_shim_read: interpolation needs the hamming84 codec");
  if (out_dtype < KVECC_F32 || out_dtype > KVECC_BF16)
    return set_error(KVECC_EINVAL, "cpu_shim_read: bad dtype %d", out_dtype);
  if (num_layers < 1 || block_size < 1 || layer < 0 || layer >= num_layers)
    return set_error(KVECC_EINVAL, "cpu_shim_read: bad cache geometry");
  if (!k_cache || !v_cache || !k_scales || !v_scales || !block_table || !k_out || !v_out)
    return set_error(KVECC_EINVAL, "cpu_shim_read: null pointer");
  static uint16_t tab[8192];
  static bool ready = [] {
    build_golay_parity_table(tab);
    build_golay_correct_table(tab + 4096);
    return true;
  }();
  (void)ready;
  const bool packed = codec == KVECC_CODEC_GOLAY_PACKED;
  const bool golay = codec == KVECC_CODEC_GOLAY || packed;
  const int64_t g = golay ? (d + 2) / 3 : d;
  auto slot_of = [&](int64_t l, int64_t h) {
    return (((int64_t)block_table[l / block_size] * num_layers + layer) * hkv + h) * block_size +
           l % block_size;
  };
  const int64_t per_side = hkv * ctx;
  const std::vector<uint8_t> zero_row(golay ? 0 : (size_t)d, 0);  // a missing block's codewords
  std::vector<Acc2> acc(std::max(1, clamp_threads(threads, 2 * per_side, 1)));
  parallel_for(2 * per_side, threads, 1, [&](int64_t b, int64_t e, int t) {
    uint32_t n1 = 0, n2 = 0;
    uint64_t bits = 0, unc = 0;
    for (int64_t item = b; item < e; ++item) {
      const int side = (int)(item / per_side);
      const int64_t hl = item - side * per_side;
      const int64_t h = hl / ctx, l = hl % ctx;
      const int64_t slot = slot_of(l, h);
      void *out = side ? v_out : k_out;
      const int64_t o = (h * ctx + l) * d;
      if (block_table[l / block_size] < 0) {  // no physical block: zeros
        for (int64_t j = 0; j < d; ++j) store_y(out, out_dtype, o + j, 0.0f);
        continue;
      }
      const float s = (side ? v_scales : k_scales)[slot];
      if (golay) {
        const void *cache = side ? v_cache : k_cache;
        for (int64_t q = 0; q < g; ++q) {
          uint32_t cnt, w;
          if (packed) {
            const uint8_t *c = reinterpret_cast<const uint8_t *>(cache) + slot * KVECC_GOLAY_PACKED_ROW(g) + 3 * q;
            w = (uint32_t)c[0] | (uint32_t)c[1] << 8 | (uint32_t)c[2] << 16;
          } else {
            w = (uint32_t)reinterpret_cast<const int32_t *>(cache)[slot * g + q];
          }
          const uint32_t dw = golay_decode1(w, tab, tab + 4096, cnt);
          bits += cnt & 3u;
          unc += cnt >> 2;
          for (int64_t u = 0; u < 3 && 3 * q + u < d; ++u)
            store_y(out, out_dtype, o + 3 * q + u, ((float)(dw >> (4 * u) & 0xFu) - 8.0f) * s);
        }
        continue;
      }
      const uint8_t *base = reinterpret_cast<const uint8_t *>(side ? v_cache : k_cache);
      const uint8_t *c = base + slot * d;
      // neighbours in a missing block read as zero codewords (the device kernels do the same)
      const int64_t ll = l > 0 ? l - 1 : 0, lr = l + 1 < ctx ? l + 1 : ctx - 1;
      const uint8_t *cl = block_table[ll / block_size] < 0 ? zero_row.data() : base + slot_of(ll, h) * d;
      const uint8_t *cr = block_table[lr / block_size] < 0 ? zero_row.data() : base + slot_of(lr, h) * d;
      for (int64_t j = 0; j < d; ++j) {
        uint32_t q = c[j], type = 0;
        if (codec == KVECC_CODEC_H84) {
          h84_decode4(c[j], q, type, n1, n2);
          if (interp) {
            uint32_t ql, qr, tt, u1 = 0, u2 = 0;
            h84_decode4(cl[j], ql, tt, u1, u2);
            h84_decode4(cr[j], qr, tt, u1, u2);
            q = interp_word(q, ql, qr, type) & 0xFFu;
          }
        } else if (codec == KVECC_CODEC_H74) {
          h74_decode4(c[j], q, type, n1);
        }
        store_y(out, out_dtype, o + j, ((float)q - 8.0f) * s);
      }
    }
    acc[t].a += golay ? bits : n1;
    acc[t].b += golay ? unc : n2;
  });
  add_stats(stats, acc, 2);
  return KVECC_OK;
}

KVECC_API int kvecc_cpu_shim_read_batch(const void *k_cache, const void *v_cache,
                                        const float *k_scales, const float *v_scales,
                                        const int32_t *block_table, int64_t table_stride,
                                        int64_t batch, int64_t ctx, int64_t hkv, int64_t d,
                                        int64_t num_layers, int64_t block_size, int64_t layer,
                                        int codec, int interp, void *k_out, void *v_out,
                                        int out_dtype, uint64_t *stats, int threads) {
  if (batch < 0) return set_error(KVECC_EINVAL, "cpu_shim_read_batch: negative batch");
  if (batch > 1 && ctx > 0 && table_stride < (ctx + block_size - 1) / std::max<int64_t>(block_size, 1))
    return set_error(KVECC_EINVAL, "cpu_shim_read_batch: table stride too small");
  const int64_t osz = out_dtype == KVECC_F32 ? 4 : 2;
  for (int64_t b = 0; b < batch; ++b) {
    const int64_t off = b * hkv * ctx * d * osz;
    const int rc = kvecc_cpu_shim_read(k_cache, v_cache, k_scales, v_scales, block_table + b * table_stride,
                                       ctx, hkv, d, num_layers, block_size, layer, codec, interp,
                                       reinterpret_cast<char *>(k_out) + off,
                                       reinterpret_cast<char *>(v_out) + off, out_dtype, stats, threads);
    if (rc != KVECC_OK) return rc;
  }
  return KVECC_OK;
}

// ---- paged decode attention (host twin of attention.hip) ---------------------
// The reference's order exactly: one (b, h) at a time, tokens in order, online
// softmax in fp32 (attention_ecc.py:355-427).  No valid token: Hamming(8,4)
// -8.0 per lane (the reference kernel's -1e20 masking, :342,391-423), Golay 0
// (reference_attention_ecc, :806-807,885-886).
KVECC_API int kvecc_cpu_paged_attention(const void *query, int q_dtype, const void *k_cache,
                                        const void *v_cache, const int32_t *block_table,
                                        const int32_t *context_lens, const float *k_scales,
                                        const float *v_scales, void *out, int64_t batch,
                                        int64_t heads, int64_t kv_heads, int64_t head_dim,
                                        int64_t num_blocks, int64_t num_layers, int64_t layer, int64_t block_size,
                                        int64_t max_blocks, int64_t max_context_len,
                                        float sm_scale, int codec, int threads) {
  if (batch < 0 || heads < 0 || kv_heads < 0 || head_dim < 0)
    return set_error(KVECC_EINVAL, "cpu_paged_attention: negative size");
  if (batch == 0 || heads == 0) return KVECC_OK;
  if (kv_heads < 1 || heads % kv_heads != 0)
    return set_error(KVECC_EINVAL, "cpu_paged_attention: heads not a multiple of kv heads");
  if (head_dim < 1) return set_error(KVECC_EINVAL, "cpu_paged_attention: empty head_dim");
  if (codec != KVECC_CODEC_H84 && codec != KVECC_CODEC_GOLAY && codec != KVECC_CODEC_GOLAY_PACKED)
    return set_error(KVECC_EINVAL, "cpu_paged_attention: codec %d (hamming84 or golay only)", codec);
  if (q_dtype < KVECC_F32 || q_dtype > KVECC_BF16)
    return set_error(KVECC_EINVAL, "cpu_paged_attention: bad dtype %d", q_dtype);
  if (num_layers < 1 || layer < 0 || layer >= num_layers || block_size < 1 || max_blocks < 1)
    return set_error(KVECC_EINVAL, "cpu_paged_attention: bad cache geometry");
  if (!query || !k_cache || !v_cache || !block_table || !context_lens || !k_scales || !v_scales || !out)
    return set_error(KVECC_EINVAL, "cpu_paged_attention: null pointer");
  if (max_context_len <= 0) max_context_len = max_blocks * block_size;
  static uint16_t tab[8192];
  static bool ready = [] {
    build_golay_parity_table(tab);
    build_golay_correct_table(tab + 4096);
    return true;
  }();
  (void)ready;
  const bool packed = codec == KVECC_CODEC_GOLAY_PACKED;
  const bool golay = codec == KVECC_CODEC_GOLAY || packed;
  const int64_t g = golay ? (head_dim + 2) / 3 : head_dim;
  const int64_t groups = heads / kv_heads;
  parallel_for(batch * heads, threads, 1, [&](int64_t b0, int64_t e0, int) {
    std::vector<float> q(head_dim), kv(head_dim), acc(head_dim);
    auto decode_row = [&](const void *cache, int64_t srow, float s) {
      if (golay) {
        for (int64_t k = 0; k < g; ++k) {
          uint32_t cnt, w;
          if (packed) {
            const uint8_t *c = reinterpret_cast<const uint8_t *>(cache) + srow * KVECC_GOLAY_PACKED_ROW(g) + 3 * k;
            w = (uint32_t)c[0] | (uint32_t)c[1] << 8 | (uint32_t)c[2] << 16;
          } else {
            w = (uint32_t)reinterpret_cast<const int32_t *>(cache)[srow * g + k];
          }
          const uint32_t dw = golay_decode1(w, tab, tab + 4096, cnt);
          for (int64_t u = 0; u < 3 && 3 * k + u < head_dim; ++u)
            kv[3 * k + u] = ((float)(dw >> (4 * u) & 0xFu) - 8.0f) * s;
        }
      } else {
        const uint8_t *c = reinterpret_cast<const uint8_t *>(cache) + srow * head_dim;
        for (int64_t j = 0; j < head_dim; ++j) {
          uint32_t d, t, n1 = 0, n2 = 0;
          h84_decode4(c[j], d, t, n1, n2);
          kv[j] = ((float)d - 8.0f) * s;
        }
      }
    };
    for (int64_t bh = b0; bh < e0; ++bh) {
      const int64_t b = bh / heads, h = bh % heads, hk = h / groups;
      for (int64_t j = 0; j < head_dim; ++j) q[j] = load_x(query, q_dtype, bh * head_dim + j);
      std::fill(acc.begin(), acc.end(), 0.0f);
      float m = -INFINITY, l = 0.0f;
      const int64_t ctx = std::min<int64_t>(std::min<int64_t>(context_lens[b], max_context_len),
                                            max_blocks * block_size);
      for (int64_t pos = 0; pos < ctx; ++pos) {
        const int32_t blk = block_table[b * max_blocks + pos / block_size];
        if (blk < 0) continue;
        const int64_t srow = (((int64_t)blk * num_layers + layer) * kv_heads + hk) * block_size +
                             pos % block_size;
        decode_row(k_cache, srow, k_scales[srow]);
        float sc = 0.0f;
        for (int64_t j = 0; j < head_dim; ++j) sc += q[j] * kv[j];
        sc *= sm_scale;
        const float mn = std::max(m, sc);
        const float alpha = m == -INFINITY ? 0.0f : std::exp(m - mn);
        const float beta = std::exp(sc - mn);
        decode_row(v_cache, srow, v_scales[srow]);
        for (int64_t j = 0; j < head_dim; ++j) acc[j] = alpha * acc[j] + beta * kv[j];
        l = alpha * l + beta;
        m = mn;
      }
      for (int64_t j = 0; j < head_dim; ++j)
        store_y(out, q_dtype, bh * head_dim + j, l > 0.0f ? acc[j] / l : golay ? 0.0f : -8.0f);
    }
  });
  return KVECC_OK;
}

}  // extern "C"
