// quant.hip -- fused INT4 quantize+encode and decode+dequantize of KV rows.
//
// Reference: ecc_codecs/triton_kernels/fused_kernels.py:18-269 (quantize +
// Hamming encode) and :272-437 (Hamming(8,4) decode + dequantize), and the
// shim's torch path ecc_shim.py:572-580 with compute_quantization_scales
// (kv_cache/paged_cache_ecc.py:302-334), which is the parity target:
//   scale = absmax(row) / 7  (0 -> 1),  q = round_half_even(x / scale)
//   clamped to [-8, 7] + 8,  in fp32, the scale under the caller's rule
//   (KVECC_SCALE_*: IEEE division as torch on the CPU, or absmax * RN(1/7) as
//   torch on a GPU) and x / scale correctly rounded.
//
// gfx950 design: a row (one head vector, D values) is owned by LPR lanes of a
// wave (LPR = the power of two covering D / VEC, VEC elements = 16 B per lane
// per load), so a wave processes 64 / LPR rows at once and the absmax is a
// short __shfl_xor butterfly inside the row's lane group.  Loads are 16 B per
// lane, the 8-bit codewords leave as VEC-byte stores.
#include "kvecc_internal.h"

namespace kvecc {

// to_f32 / from_f32: kvecc_internal.h

// single-value encoder: codec_math.h encode_nibble (KVECC_CODEC_* codes)
__device__ __forceinline__ uint32_t enc_nibble(uint32_t v, int codec) { return encode_nibble(v, codec); }

__device__ __forceinline__ float row_max(float v, int lpr) {
  for (int off = lpr >> 1; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, kWave));
  return v;
}

template <typename T, int VEC>
struct alignas(sizeof(T) * VEC) Vec {
  T v[VEC];
};

// Quantize + encode. rows are contiguous of length d; lanes [g*lpr, (g+1)*lpr)
// of a wave own row (wave_row0 + g).
template <typename T, int VEC>
__global__ __launch_bounds__(kBlock) void quantize_encode_kernel(const T *__restrict__ x, int codec,
                                                                 int rule, uint8_t *__restrict__ cw,
                                                                 float *__restrict__ scales,
                                                                 int64_t rows, int64_t d, int lpr) {
  const int lane = threadIdx.x & (kWave - 1);
  const int rows_per_wave = kWave / lpr;
  const int sub = lane / lpr, li = lane % lpr;
  const int64_t waves = (int64_t)gridDim.x * (kBlock / kWave);
  const int64_t wave_id = (int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
  const int64_t nchunk = d / VEC;  // VEC divides d on this path
  for (int64_t r0 = wave_id * rows_per_wave; r0 < rows; r0 += waves * rows_per_wave) {
    const int64_t r = r0 + sub;
    const bool live = r < rows;
    const T *xr = x + r * d;
    float amax = 0.0f;
    if (live) {
      for (int64_t c = li; c < nchunk; c += lpr) {
        Vec<T, VEC> v = *reinterpret_cast<const Vec<T, VEC> *>(xr + c * VEC);
#pragma unroll
        for (int k = 0; k < VEC; ++k) amax = fmaxf(amax, fabsf(to_f32<T>(v.v[k])));
      }
    }
    amax = row_max(amax, lpr);
    const float scale = row_scale(amax, rule);
    if (!live) continue;
    if (li == 0) scales[r] = scale;
    uint8_t *cr = cw + r * d;
    for (int64_t c = li; c < nchunk; c += lpr) {
      Vec<T, VEC> v = *reinterpret_cast<const Vec<T, VEC> *>(xr + c * VEC);
      Vec<uint8_t, VEC> o;
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        float q = rintf(__fdiv_rn(to_f32<T>(v.v[k]), scale));
        q = fminf(fmaxf(q, -8.0f), 7.0f);
        o.v[k] = (uint8_t)enc_nibble((uint32_t)(int)(q + 8.0f), codec);
      }
      *reinterpret_cast<Vec<uint8_t, VEC> *>(cr + c * VEC) = o;
    }
  }
}

// Rows of at most 64 chunks (every row of the shim and the reference's tests):
// each lane loads its one 16-byte chunk ONCE, non-temporally, on a full grid of
// wave tiles -- a wave owns kQeTile row groups (64 / LPR rows each), issues all
// their loads first, then quantizes and encodes them, and workgroups retire
// instead of striding.  fp16 D=128 rows: 71.2 -> 63.2 us against round 4's
// grid-strided one-group-per-iteration kernel (64 workgroups per CU), 77.6 with
// one group per wave (profiles/r05/exp_r05e.log quant_fp16 v0-v3; 4 groups per
// wave 63.2 as well).
constexpr int kQeTile = 2;
template <typename T, int VEC, int LPR>
__global__ __launch_bounds__(kBlock) void quantize_encode_tile_kernel(const T *__restrict__ x, int codec,
                                                                      int rule, uint8_t *__restrict__ cw,
                                                                      float *__restrict__ scales,
                                                                      int64_t rows, int64_t d) {
  static_assert(sizeof(T) * VEC == 16, "one 16-byte chunk per lane");
  constexpr int rows_per_wave = kWave / LPR;
  const int lane = threadIdx.x & (kWave - 1);
  const int sub = lane / LPR, li = lane % LPR;
  const int64_t nchunk = d / VEC;
  const int64_t wave_id = (int64_t)blockIdx.x * (kBlock / kWave) + threadIdx.x / kWave;
  const int64_t r0 = wave_id * rows_per_wave * kQeTile + sub;
  Vec<T, VEC> v[kQeTile];
  bool live[kQeTile];
#pragma unroll
  for (int u = 0; u < kQeTile; ++u) {
    const int64_t r = r0 + u * rows_per_wave;
    live[u] = r < rows && li < nchunk;
    if (live[u]) {
      const u32x4 raw = ld_stream(reinterpret_cast<const u32x4 *>(x + r * d + li * VEC));
      __builtin_memcpy(&v[u], &raw, 16);
    }
  }
#pragma unroll
  for (int u = 0; u < kQeTile; ++u) {
    const int64_t r = r0 + u * rows_per_wave;
    float f[VEC];
    float amax = 0.0f;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      f[k] = live[u] ? to_f32<T>(v[u].v[k]) : 0.0f;
      amax = fmaxf(amax, fabsf(f[k]));
    }
    amax = group_max_nonneg<LPR>(amax);
    const float scale = row_scale(amax, rule);
    if (!live[u]) continue;
    if (li == 0) scales[r] = scale;
    // x / scale: reciprocal + FMA correction for 16-bit inputs (codec_math.h
    // div_recip, exhaustively checked), IEEE division otherwise
    uint32_t nq[VEC];
    if (sizeof(T) == 2 && recip_ok(scale)) {
      const float inv = div_rn(1.0f, scale);
#pragma unroll
      for (int k = 0; k < VEC; ++k) nq[k] = nibble_of_quotient(div_recip(f[k], scale, inv));
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k) nq[k] = quantize_nibble(f[k], scale);
    }
    // four quantized nibbles per word, encoded SWAR (codec_math.h)
    uint32_t wds[VEC / 4];
#pragma unroll
    for (int k = 0; k < VEC / 4; ++k) {
      uint32_t wq = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) wq |= nq[4 * k + e] << (8 * e);
      wds[k] = codec == KVECC_CODEC_H84 ? h84_encode4(wq)
               : codec == KVECC_CODEC_H74 ? h74_encode4(wq)
                                          : wq;
    }
    if (VEC == 8) {
      uint64_t bits = (uint64_t)wds[0] | (uint64_t)wds[VEC / 4 - 1] << 32;
      st_stream(reinterpret_cast<uint64_t *>(cw + r * d + li * VEC), bits);
    } else {
      st_stream(reinterpret_cast<uint32_t *>(cw + r * d + li * VEC), wds[0]);
    }
  }
}

// Hamming(8,4) decode of one codeword byte: data, type (codec_math.h h84_decode4)
__device__ __forceinline__ uint32_t dec84(uint32_t c, uint32_t &type) {
  uint32_t data, n1 = 0, n2 = 0;
  h84_decode4(c & 0xFFu, data, type, n1, n2);
  return data;
}

template <typename TO, int VEC>
__global__ __launch_bounds__(kBlock) void decode_dequant_kernel(const uint8_t *__restrict__ cw,
                                                                const float *__restrict__ scales,
                                                                TO *__restrict__ out, int64_t rows,
                                                                int64_t d, int zero_doubles,
                                                                uint64_t *__restrict__ stats) {
  const int64_t nchunk = d / VEC;
  const int64_t total = rows * nchunk;
  uint32_t n1 = 0, n2 = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    const int64_t r = i / nchunk;
    const float s = scales[r];
    Vec<uint8_t, VEC> c = *reinterpret_cast<const Vec<uint8_t, VEC> *>(cw + i * VEC);
    Vec<TO, VEC> o;
#pragma unroll
    for (int k = 0; k < VEC; ++k) {
      uint32_t t;
      uint32_t q = dec84(c.v[k], t);
      if (zero_doubles && t == 2) q = 0;
      n1 += t == 1;
      n2 += t == 2;
      o.v[k] = from_f32<TO>(dequant1(q, s));
    }
    *reinterpret_cast<Vec<TO, VEC> *>(out + i * VEC) = o;
  }
  if (stats) flush_stats2(stats, n1, n2);
}

// Wave tiles: a wave owns T x 64 consecutive 16-byte output vectors (fp16 /
// bf16: 8 codewords per vector, T = 4; fp32: 4 codewords, T = 2); load u and
// store u of every lane cover one contiguous span (512 / 256 B of codewords,
// 1 KiB of output) and the grid is full, so each wave writes T KiB and
// retires.  At [8*4096*32, 128] (tools/exp/run_r05.py, profiles/r05/exp_r05.log)
// fp16 66.2 vs 68.9 us for the grid-strided kernel (1 vector per wave: 83.9),
// fp32 107.3 vs 119.7 (T = 4 / 8: 109.3 / 110.9).  Row scales: a shift when
// the vectors per row are a power of two, else a 32-bit division.
template <typename TO>
constexpr int kDdTile = sizeof(TO) == 4 ? 2 : 4;
template <typename TO>
__global__ __launch_bounds__(kBlock) void decode_dequant_tile_kernel(const void *__restrict__ cwv,
                                                                     const float *__restrict__ scales,
                                                                     u32x4 *__restrict__ out, uint32_t nchunk,
                                                                     int shift, uint32_t total, int zero_doubles,
                                                                     uint64_t *__restrict__ stats) {
  constexpr int T = kDdTile<TO>, kW = 4 / (int)sizeof(TO);  // codeword words per vector
  using InT = typename std::conditional<kW == 1, uint32_t, u32x2>::type;
  const InT *cw = reinterpret_cast<const InT *>(cwv);
  const uint32_t lane = threadIdx.x & (kWave - 1);
  const uint32_t wave = (blockIdx.x * kBlock + threadIdx.x) / kWave;
  const uint32_t base = wave * (kWave * T) + lane;
  uint32_t n1 = 0, n2 = 0;
  InT w[T];
  float s[T];
#pragma unroll
  for (int u = 0; u < T; ++u) {
    const uint32_t i = base + u * kWave;
    w[u] = i < total ? ld_stream(cw + i) : InT{};  // codeword 0: no error counted
    s[u] = i < total ? scales[shift >= 0 ? i >> shift : i / nchunk] : 0.0f;
  }
#pragma unroll
  for (int u = 0; u < T; ++u) {
    const uint32_t i = base + u * kWave;
    uint32_t wd[kW], nb[2] = {0u, 0u};
    __builtin_memcpy(wd, &w[u], sizeof(wd));
#pragma unroll
    for (int k = 0; k < kW; ++k) {
      uint32_t q, t;
      h84_decode4(wd[k], q, t, n1, n2);
      if (zero_doubles) {  // double errors -> data 0 (fused_kernels.py:344)
        const uint32_t dbl = (t >> 1) & ~t & 0x01010101u;
        q &= ~(dbl * 0xFFu);
      }
      nb[k] = q;
    }
    if (i < total) st_stream(out + i, dq16<TO>(nb, s[u], false));
  }
  if (stats) flush_stats2(stats, n1, n2);
}

static int lanes_per_row(int64_t chunks) {
  int l = 1;
  while (l < chunks && l < kWave) l <<= 1;
  return l;
}

template <typename T>
static void launch_qe(const void *x, int codec, int rule, uint8_t *cw, float *scales, int64_t rows,
                      int64_t d, hipStream_t st) {
  constexpr int V = 16 / sizeof(T);
  const T *xt = reinterpret_cast<const T *>(x);
  bool vec = d % V == 0 && aligned(x, 16) && aligned(cw, V);
  if (vec && d / V <= kWave) {
    const int lpr = lanes_per_row(d / V);
    const int64_t waves = cdiv(rows, (int64_t)(kWave / lpr) * kQeTile);
    const unsigned grid = (unsigned)cdiv(waves, kBlock / kWave);
#define KVECC_QE1C(L)                                                                           \
  case L:                                                                                       \
    KVECC_LAUNCH((quantize_encode_tile_kernel<T, V, L>), dim3(grid), dim3(kBlock), 0, st, xt, \
                 codec, rule, cw, scales, rows, d);                                             \
    break;
    switch (lpr) {
      KVECC_QE1C(1) KVECC_QE1C(2) KVECC_QE1C(4) KVECC_QE1C(8) KVECC_QE1C(16) KVECC_QE1C(32)
      KVECC_QE1C(64)
    }
#undef KVECC_QE1C
  } else if (vec) {
    int lpr = lanes_per_row(d / V);
    int64_t waves = cdiv(rows, kWave / lpr);
    KVECC_LAUNCH((quantize_encode_kernel<T, V>), dim3(grid_for(waves, kBlock / kWave)),
                       dim3(kBlock), 0, st, xt, codec, rule, cw, scales, rows, d, lpr);
  } else {
    int lpr = lanes_per_row(d);
    int64_t waves = cdiv(rows, kWave / lpr);
    KVECC_LAUNCH((quantize_encode_kernel<T, 1>), dim3(grid_for(waves, kBlock / kWave)),
                       dim3(kBlock), 0, st, xt, codec, rule, cw, scales, rows, d, lpr);
  }
}

template <typename TO>
static void launch_dd(const uint8_t *cw, const float *scales, void *out, int64_t rows, int64_t d,
                      int zero_doubles, uint64_t *stats, hipStream_t st) {
  TO *o = reinterpret_cast<TO *>(out);
  constexpr int kCw = 16 / sizeof(TO);  // codewords per 16-byte output vector
  if (d % kCw == 0 && aligned(cw, kCw) && aligned(out, 16) && rows * d < 0xFFFFFFFFLL) {
    const uint32_t total = (uint32_t)(rows * (d / kCw));
    const uint32_t nchunk = (uint32_t)(d / kCw);
    const int shift = (nchunk & (nchunk - 1)) == 0 ? __builtin_ctz(nchunk) : -1;
    // full-grid wave tiles (decode_dequant_tile_kernel)
    KVECC_LAUNCH((decode_dequant_tile_kernel<TO>), dim3((unsigned)cdiv(total, (int64_t)kBlock * kDdTile<TO>)),
                 dim3(kBlock), 0, st, cw, scales, reinterpret_cast<u32x4 *>(out), nchunk, shift, total,
                 zero_doubles, stats);
  } else if (d % 4 == 0 && aligned(cw, 4) && aligned(out, 4 * sizeof(TO))) {
    int64_t total = rows * (d / 4);
    KVECC_LAUNCH((decode_dequant_kernel<TO, 4>), dim3(grid_for(total, kBlock)), dim3(kBlock),
                       0, st, cw, scales, o, rows, d, zero_doubles, stats);
  } else {
    int64_t total = rows * d;
    KVECC_LAUNCH((decode_dequant_kernel<TO, 1>), dim3(grid_for(total, kBlock)), dim3(kBlock),
                       0, st, cw, scales, o, rows, d, zero_doubles, stats);
  }
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_quantize_encode_rows(const void *x, int x_dtype, int codec, int scale_rule,
                                         uint8_t *cw, float *scales, int64_t rows, int64_t d,
                                         void *stream) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "quantize_encode_rows: negative size");
  if (rows == 0) return KVECC_OK;
  if (d == 0) return set_error(KVECC_EINVAL, "quantize_encode_rows: empty rows");
  if (!x || !cw || !scales) return set_error(KVECC_EINVAL, "quantize_encode_rows: null pointer");
  if (codec != KVECC_CODEC_NONE && codec != KVECC_CODEC_H74 && codec != KVECC_CODEC_H84)
    return set_error(KVECC_EINVAL, "quantize_encode_rows: bad codec %d", codec);
  if (scale_rule != KVECC_SCALE_DIV7 && scale_rule != KVECC_SCALE_MUL_INV7)
    return set_error(KVECC_EINVAL, "quantize_encode_rows: bad scale rule %d", scale_rule);
  hipStream_t st = as_stream(stream);
  switch (x_dtype) {
    case KVECC_F32: launch_qe<float>(x, codec, scale_rule, cw, scales, rows, d, st); break;
    case KVECC_F16: launch_qe<__half>(x, codec, scale_rule, cw, scales, rows, d, st); break;
    case KVECC_BF16: launch_qe<__hip_bfloat16>(x, codec, scale_rule, cw, scales, rows, d, st); break;
    default: return set_error(KVECC_EINVAL, "quantize_encode_rows: bad dtype %d", x_dtype);
  }
  return check_launch("quantize_encode_rows");
}

KVECC_API int kvecc_decode_dequant_h84_rows(const uint8_t *cw, const float *scales, void *out,
                                            int out_dtype, int64_t rows, int64_t d,
                                            int zero_doubles, uint64_t *stats, void *stream) {
  if (rows < 0 || d < 0) return set_error(KVECC_EINVAL, "decode_dequant_h84_rows: negative size");
  if (rows == 0 || d == 0) return KVECC_OK;
  if (!cw || !scales || !out) return set_error(KVECC_EINVAL, "decode_dequant_h84_rows: null pointer");
  hipStream_t st = as_stream(stream);
  switch (out_dtype) {
    case KVECC_F32: launch_dd<float>(cw, scales, out, rows, d, zero_doubles, stats, st); break;
    case KVECC_F16: launch_dd<__half>(cw, scales, out, rows, d, zero_doubles, stats, st); break;
    case KVECC_BF16: launch_dd<__hip_bfloat16>(cw, scales, out, rows, d, zero_doubles, stats, st); break;
    default: return set_error(KVECC_EINVAL, "decode_dequant_h84_rows: bad dtype %d", out_dtype);
  }
  return check_launch("decode_dequant_h84_rows");
}

}  // extern "C"
