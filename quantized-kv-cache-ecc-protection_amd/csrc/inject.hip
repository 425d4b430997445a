// inject.hip -- bit-exact Bernoulli bit-flip fault injection.
//
// Reference: ecc_codecs/triton_kernels/fault_injection_triton.py:228-334
// (per-bit tl.rand) and :57-224 (rand4x), with Triton's Philox4x32-10 and
// uint->float mapping (triton/language/random.py:12-143).
//
// For element `off` of an N-element tensor and bit b the reference draws
//   key = int32(seed * (N * n_bits) + off * n_bits + b)   (sign-extended to 64)
//   c0  = Philox4x32-10(counter = (off, 0, 0, 0), key).word0
//   u   = fp32(fold(int32 c0)) * 0x2FFFFFFF,  fold(x) = x < 0 ? -x-1 : x
//   flip iff u < fp32(ber)
// Both roundings are monotone, so `u < ber` is exactly `fold(c0) < T` for an
// integer threshold T found on the host (kvecc_ber_threshold): the kernel
// compares integers, no int->float conversion or multiply.
//
// The kernels are VALU-bound (one Philox = 10 rounds of 2 32x32->64 products
// per bit); each lane handles 4 consecutive elements so that round 1 of all
// their bits shares the counter products, and the loads/stores stay 4-16 B.
#include "kvecc_internal.h"

namespace kvecc {

// Philox rounds, the integer BER test and the per-element flip masks live in
// codec_math.h (shared with the host backend).
template <int NB>
__device__ __forceinline__ uint32_t flip_mask(uint32_t key_base, uint32_t ctr, uint32_t thr,
                                              int nb_rt) {
  return philox_flip_mask<NB>(key_base, ctr, thr, nb_rt);
}

struct InjectArgs {
  int64_t n;         // elements in this call
  int64_t offset0;   // global index of element 0
  uint32_t seedmul;  // (seed * global_n * n_bits) mod 2^32
  uint32_t nbits;    // n_bits as the reference uses it in the key
  uint32_t thr;      // integer BER threshold
  int nb_eff;        // bits actually drawn (runtime form)
};

// 4 elements per lane; T = uint8_t or int32_t
template <typename T, int NB, bool COUNTS, bool STATS>
__global__ __launch_bounds__(kBlock) void inject_kernel(const T *in, T *out,
                                                        uint8_t *__restrict__ counts, InjectArgs a,
                                                        uint64_t *__restrict__ stats) {
  uint32_t flips = 0, hit = 0;
  const int64_t ngroups = (a.n + 3) / 4;
  for (int64_t gi = (int64_t)blockIdx.x * kBlock + threadIdx.x; gi < ngroups;
       gi += (int64_t)gridDim.x * kBlock) {
    const int64_t i0 = gi * 4;
    const bool full = i0 + 4 <= a.n;
    T v[4];
    if (full && sizeof(T) == 1) {
      uint32_t w = *reinterpret_cast<const uint32_t *>(in + i0);  // host checked 4-B alignment
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = (T)(w >> (8 * k));
    } else if (full) {
      u32x4 w = *reinterpret_cast<const u32x4 *>(in + i0);  // host checked 16-B alignment
      v[0] = (T)w.x; v[1] = (T)w.y; v[2] = (T)w.z; v[3] = (T)w.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = i0 + k < a.n ? in[i0 + k] : (T)0;
    }
    uint32_t cnt[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t g = (uint32_t)(a.offset0 + i0 + k);  // global element index (int32 counter)
      const uint32_t m = flip_mask<NB>(a.seedmul + g * a.nbits, g, a.thr, a.nb_eff);
      v[k] = (T)((uint32_t)v[k] ^ m);
      cnt[k] = __builtin_popcount(m);
      if (STATS && i0 + k < a.n) {
        flips += cnt[k];
        hit += cnt[k] != 0;
      }
    }
    if (full && sizeof(T) == 1) {
      uint32_t w = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) w |= ((uint32_t)v[k] & 0xFFu) << (8 * k);
      *reinterpret_cast<uint32_t *>(out + i0) = w;
    } else if (full) {
      u32x4 w;
      w.x = (uint32_t)v[0]; w.y = (uint32_t)v[1]; w.z = (uint32_t)v[2]; w.w = (uint32_t)v[3];
      *reinterpret_cast<u32x4 *>(out + i0) = w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (i0 + k < a.n) out[i0 + k] = v[k];
    }
    if (COUNTS) {
      if (full) {
        *reinterpret_cast<uint32_t *>(counts + i0) = cnt[0] | cnt[1] << 8 | cnt[2] << 16 | cnt[3] << 24;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (i0 + k < a.n) counts[i0 + k] = (uint8_t)cnt[k];
      }
    }
  }
  if (STATS) flush_stats2(stats, flips, hit);
}

// scalar variant for unaligned buffers: one element per lane
template <typename T, int NB>
__global__ __launch_bounds__(kBlock) void inject_scalar_kernel(const T *in,
                                                               T *out,
                                                               uint8_t *__restrict__ counts,
                                                               InjectArgs a,
                                                               uint64_t *__restrict__ stats) {
  uint32_t flips = 0, hit = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < a.n;
       i += (int64_t)gridDim.x * kBlock) {
    const uint32_t g = (uint32_t)(a.offset0 + i);
    const uint32_t m = flip_mask<NB>(a.seedmul + g * a.nbits, g, a.thr, a.nb_eff);
    out[i] = (T)((uint32_t)in[i] ^ m);
    uint32_t c = __builtin_popcount(m);
    if (counts) counts[i] = (uint8_t)c;
    flips += c;
    hit += c != 0;
  }
  if (stats) flush_stats2(stats, flips, hit);
}

// per-row scheme: row r has its own seed (seed_base + r) and N = row_len
struct RowArgs {
  int64_t rows, row_len;
  uint32_t seed_base;
  uint32_t rowmul;  // (row_len * n_bits) mod 2^32
  uint32_t nbits, thr;
  int nb_eff;
};

template <typename T, int NB>
__global__ __launch_bounds__(kBlock) void inject_rows_kernel(const T *in,
                                                             T *out, RowArgs a,
                                                             uint64_t *__restrict__ stats) {
  uint32_t flips = 0, hit = 0;
  const int64_t total = a.rows * a.row_len;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / a.row_len;
    const uint32_t j = (uint32_t)(i - r * a.row_len);
    const uint32_t seed = a.seed_base + (uint32_t)r;
    const uint32_t m = flip_mask<NB>(seed * a.rowmul + j * a.nbits, j, a.thr, a.nb_eff);
    out[i] = (T)((uint32_t)in[i] ^ m);
    uint32_t c = __builtin_popcount(m);
    flips += c;
    hit += c != 0;
  }
  if (stats) flush_stats2(stats, flips, hit);
}

// rand4x variants: batch k of 4 bits uses key seed*N + off + k*N and words c0..c3
template <typename T>
__global__ __launch_bounds__(kBlock) void inject_vec_kernel(const T *in,
                                                            T *out,
                                                            uint8_t *__restrict__ counts,
                                                            int64_t n, uint32_t seedn,
                                                            uint32_t nn, uint32_t thr, int nb,
                                                            uint64_t *__restrict__ stats) {
  uint32_t flips = 0, hit = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    const uint32_t m = philox_flip_mask_vec(seedn, nn, (uint32_t)i, thr, nb);
    out[i] = (T)((uint32_t)in[i] ^ m);
    uint32_t c = __builtin_popcount(m);
    if (counts) counts[i] = (uint8_t)c;
    flips += c;
    hit += c != 0;
  }
  if (stats) flush_stats2(stats, flips, hit);
}

template <typename T, int NB>
static void launch_flat(const T *in, T *out, uint8_t *counts, const InjectArgs &a,
                        uint64_t *stats, hipStream_t st) {
  const bool vec_ok = (sizeof(T) == 1 ? (aligned(in, 4) && aligned(out, 4))
                                      : (aligned(in, 16) && aligned(out, 16))) &&
                      (!counts || aligned(counts, 4));
  if (vec_ok) {
    unsigned g = grid_for((a.n + 3) / 4, kBlock, 16);
    if (counts && stats)
      KVECC_LAUNCH((inject_kernel<T, NB, true, true>), dim3(g), dim3(kBlock), 0, st, in, out, counts, a, stats);
    else if (counts)
      KVECC_LAUNCH((inject_kernel<T, NB, true, false>), dim3(g), dim3(kBlock), 0, st, in, out, counts, a, stats);
    else if (stats)
      KVECC_LAUNCH((inject_kernel<T, NB, false, true>), dim3(g), dim3(kBlock), 0, st, in, out, counts, a, stats);
    else
      KVECC_LAUNCH((inject_kernel<T, NB, false, false>), dim3(g), dim3(kBlock), 0, st, in, out, counts, a, stats);
  } else {
    unsigned g = grid_for(a.n, kBlock, 16);
    KVECC_LAUNCH((inject_scalar_kernel<T, NB>), dim3(g), dim3(kBlock), 0, st, in, out, counts, a, stats);
  }
}

static inline uint32_t mul_wrap(int64_t a, int64_t b) {
  return (uint32_t)((uint64_t)a * (uint64_t)b);
}

template <typename T>
static int inject_flat(const T *in, T *out, uint8_t *counts, int64_t n, int n_bits, int64_t seed,
                       float ber, int64_t global_n, int64_t offset0, uint64_t *stats,
                       void *stream, const char *name) {
  if (n < 0 || global_n < 0 || offset0 < 0)
    return set_error(KVECC_EINVAL, "%s: negative size/offset", name);
  if (n == 0) return KVECC_OK;
  if (!in || !out) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  if (offset0 + n > global_n)
    return set_error(KVECC_EINVAL, "%s: shard [%lld,%lld) exceeds global_n %lld", name,
                     (long long)offset0, (long long)(offset0 + n), (long long)global_n);
  InjectArgs a;
  a.n = n;
  a.offset0 = offset0;
  a.seedmul = mul_wrap(seed, (int64_t)mul_wrap(global_n, n_bits));
  a.nbits = (uint32_t)n_bits;
  a.thr = kvecc_ber_threshold(ber);
  hipStream_t st = as_stream(stream);
  if (sizeof(T) == 1) {
    a.nb_eff = n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits);  // bit 0 is always drawn (:249-252)
    switch (a.nb_eff) {
      case 4: launch_flat<T, 4>(in, out, counts, a, stats, st); break;
      case 7: launch_flat<T, 7>(in, out, counts, a, stats, st); break;
      case 8: launch_flat<T, 8>(in, out, counts, a, stats, st); break;
      default: launch_flat<T, -1>(in, out, counts, a, stats, st); break;
    }
  } else {
    a.nb_eff = n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits);  // range(24) loop (:324-325)
    switch (a.nb_eff) {
      case 24: launch_flat<T, 24>(in, out, counts, a, stats, st); break;
      default: launch_flat<T, -1>(in, out, counts, a, stats, st); break;
    }
  }
  return check_launch(name);
}

template <typename T>
static int inject_rows(const T *in, T *out, int64_t rows, int64_t row_len, int n_bits,
                       int64_t seed_base, float ber, uint64_t *stats, void *stream,
                       const char *name) {
  if (rows < 0 || row_len < 0) return set_error(KVECC_EINVAL, "%s: negative size", name);
  if (rows == 0 || row_len == 0) return KVECC_OK;
  if (!in || !out) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  RowArgs a;
  a.rows = rows;
  a.row_len = row_len;
  a.seed_base = (uint32_t)(uint64_t)seed_base;
  a.rowmul = mul_wrap(row_len, n_bits);
  a.nbits = (uint32_t)n_bits;
  a.thr = kvecc_ber_threshold(ber);
  if (sizeof(T) == 1)
    a.nb_eff = n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits);
  else
    a.nb_eff = n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits);
  hipStream_t st = as_stream(stream);
  unsigned g = grid_for(rows * row_len, kBlock, 16);
  switch (sizeof(T) == 1 ? a.nb_eff : (a.nb_eff == 24 ? 24 : -1)) {
    case 4: KVECC_LAUNCH((inject_rows_kernel<T, 4>), dim3(g), dim3(kBlock), 0, st, in, out, a, stats); break;
    case 7: KVECC_LAUNCH((inject_rows_kernel<T, 7>), dim3(g), dim3(kBlock), 0, st, in, out, a, stats); break;
    case 8: KVECC_LAUNCH((inject_rows_kernel<T, 8>), dim3(g), dim3(kBlock), 0, st, in, out, a, stats); break;
    case 24: KVECC_LAUNCH((inject_rows_kernel<T, 24>), dim3(g), dim3(kBlock), 0, st, in, out, a, stats); break;
    default: KVECC_LAUNCH((inject_rows_kernel<T, -1>), dim3(g), dim3(kBlock), 0, st, in, out, a, stats); break;
  }
  return check_launch(name);
}

template <typename T>
static int inject_vec(const T *in, T *out, uint8_t *counts, int64_t n, int n_bits, int64_t seed,
                      float ber, uint64_t *stats, void *stream, const char *name) {
  if (n < 0) return set_error(KVECC_EINVAL, "%s: negative n", name);
  if (n == 0) return KVECC_OK;
  if (!in || !out) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  int nb = sizeof(T) == 1 ? (n_bits < 1 ? 1 : (n_bits > 8 ? 8 : n_bits))
                          : (n_bits < 0 ? 0 : (n_bits > 24 ? 24 : n_bits));
  unsigned g = grid_for(n, kBlock, 16);
  KVECC_LAUNCH(inject_vec_kernel<T>, dim3(g), dim3(kBlock), 0, as_stream(stream), in, out,
                     counts, n, mul_wrap(seed, n), (uint32_t)n, kvecc_ber_threshold(ber), nb, stats);
  return check_launch(name);
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_inject_u8(const uint8_t *in, uint8_t *out, uint8_t *counts, int64_t n,
                              int n_bits, int64_t seed, float ber, int64_t global_n,
                              int64_t offset0, uint64_t *stats, void *stream) {
  return inject_flat<uint8_t>(in, out, counts, n, n_bits, seed, ber, global_n, offset0, stats,
                              stream, "inject_u8");
}

KVECC_API int kvecc_inject_i32(const int32_t *in, int32_t *out, uint8_t *counts, int64_t n,
                               int n_bits, int64_t seed, float ber, int64_t global_n,
                               int64_t offset0, uint64_t *stats, void *stream) {
  return inject_flat<int32_t>(in, out, counts, n, n_bits, seed, ber, global_n, offset0, stats,
                              stream, "inject_i32");
}

KVECC_API int kvecc_inject_u8_vectorized(const uint8_t *in, uint8_t *out, uint8_t *counts,
                                         int64_t n, int n_bits, int64_t seed, float ber,
                                         uint64_t *stats, void *stream) {
  return inject_vec<uint8_t>(in, out, counts, n, n_bits, seed, ber, stats, stream,
                             "inject_u8_vectorized");
}

KVECC_API int kvecc_inject_i32_vectorized(const int32_t *in, int32_t *out, uint8_t *counts,
                                          int64_t n, int n_bits, int64_t seed, float ber,
                                          uint64_t *stats, void *stream) {
  return inject_vec<int32_t>(in, out, counts, n, n_bits, seed, ber, stats, stream,
                             "inject_i32_vectorized");
}

KVECC_API int kvecc_inject_rows_u8(const uint8_t *in, uint8_t *out, int64_t rows, int64_t row_len,
                                   int n_bits, int64_t seed_base, float ber, uint64_t *stats,
                                   void *stream) {
  return inject_rows<uint8_t>(in, out, rows, row_len, n_bits, seed_base, ber, stats, stream,
                              "inject_rows_u8");
}

KVECC_API int kvecc_inject_rows_i32(const int32_t *in, int32_t *out, int64_t rows,
                                    int64_t row_len, int n_bits, int64_t seed_base, float ber,
                                    uint64_t *stats, void *stream) {
  return inject_rows<int32_t>(in, out, rows, row_len, n_bits, seed_base, ber, stats, stream,
                              "inject_rows_i32");
}

}  // extern "C"
