// montecarlo.hip -- one Monte-Carlo fault-injection trial per launch.
//
// The codec-level sweep (BASELINE config 5; the reference's trial is
// encode -> inject_bit_errors_triton -> decode, e.g.
// evaluation/experiments/quantization_ecc_comparison.py:164-203 over
// evaluation/sweep.py:352-626) keeps only counters.  Run kernel by kernel it
// writes and re-reads the codewords, the decoded values and the error types
// (~1 GB of HBM traffic per trial) and issues a dozen launches; here one
// kernel reads the ground truth once and keeps everything else in registers:
//
//   x (uint8 nibbles) -> encode -> Philox flips (per bit, the reference's
//   stream: fault_injection_triton.py:228-334) -> decode -> [interpolate]
//   -> compare with x -> 5 counters (include/kvecc.h kvecc_mc_trial)
//
// The trial is VALU-bound by construction: 7-24 Philox4x32-10 evaluations per
// value or codeword (~61 VALU instructions each) against 1-3 bytes of HBM.
// The per-element arithmetic is codec_math.h's, the same functions the
// individual kernels and the host twin use.
//
// Interpolation (hamming84 + interp) needs the decoded values of the sequence
// neighbours: a lane walks a 4-value column chunk down a strip of kMcStrip
// consecutive positions with the previous, current and next decoded rows in
// registers; a strip edge's outer neighbour is recomputed (its 4 values
// encoded, flipped and decoded again) only when the edge row holds a double
// error, which at the sweep's BERs is rare.
#include "kvecc_internal.h"

namespace kvecc {

constexpr int kMcStrip = 32;   // positions per lane (interpolating trial)
constexpr int kMcPerCu = 16;   // workgroups per CU (grid-strided, as the injection)

struct McArgs {
  const uint8_t *x;
  int64_t outer, len, inner, head_dim, g;  // g = codewords per head row (Golay)
  int64_t offset0;                         // global index of the shard's first value / codeword
  uint32_t seedmul;                        // seed * global_n * n_bits (mod 2^32)
  uint32_t nbits, thr;
  uint64_t *stats;
};

// per byte of a ^ b: 1 if non-zero (interp.hip ne_bytes)
__device__ __forceinline__ uint32_t mc_ne_bytes(uint32_t x) {
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return __builtin_popcount(x & 0x01010101u);
}

// 4 consecutive values (one word of nibble bytes) at global index g0:
// encode, flip, return the noisy codeword bytes; flips / affected counted
template <bool H84, int NB>
__device__ __forceinline__ uint32_t mc_noisy4(uint32_t xw, uint32_t g0, const McArgs &a, uint32_t &flips,
                                              uint32_t &affected, uint32_t valid) {
  uint32_t cw = H84 ? h84_encode4(xw) : h74_encode4(xw);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t g = g0 + (uint32_t)k;
    uint32_t m = philox_flip_mask<NB>(a.seedmul + g * a.nbits, g, a.thr, NB);
    m = k < (int)valid ? m : 0u;
    cw ^= m << (8 * k);
    flips += __builtin_popcount(m);
    affected += m != 0;
  }
  return cw;
}

// Hamming(7,4) / (8,4) trial: 4 values per lane
template <bool H84, int NB>
__global__ __launch_bounds__(kBlock) void mc_hamming_kernel(McArgs a) {
  uint32_t c[5] = {0, 0, 0, 0, 0};  // flips, affected, corrected, detected, mismatches
  const int64_t n = a.outer * a.len * a.inner;
  const int64_t groups = (n + 3) / 4;
  for (int64_t gi = (int64_t)blockIdx.x * kBlock + threadIdx.x; gi < groups;
       gi += (int64_t)gridDim.x * kBlock) {
    const int64_t i0 = gi * 4;
    const uint32_t valid = (uint32_t)min<int64_t>(4, n - i0);
    uint32_t xw = 0;
    if (valid == 4) {
      xw = *reinterpret_cast<const uint32_t *>(a.x + i0);  // host checked 4-B alignment
    } else {
      for (uint32_t k = 0; k < valid; ++k) xw |= (uint32_t)a.x[i0 + k] << (8 * k);
    }
    const uint32_t keep = valid == 4 ? ~0u : (1u << (8 * valid)) - 1u;
    const uint32_t cw = mc_noisy4<H84, NB>(xw, (uint32_t)(a.offset0 + i0), a, c[0], c[1], valid);
    uint32_t data, t, n1 = 0, n2 = 0;
    if (H84) {
      h84_decode4(cw, data, t, n1, n2);
      // statistics of the valid values only (the padding bytes encode 0: no error)
      c[2] += n1;
      c[3] += n2;
    } else {
      h74_decode4(cw, data, t, n1);
      c[2] += n1;
    }
    c[4] += mc_ne_bytes((data ^ xw) & keep);
  }
  flush_stats_n<5>(a.stats, c);
}

// Hamming(8,4) + double-error interpolation along `len`: a lane owns the 4-value
// column chunk c4 of positions [l0, l0 + kMcRows) of sequence o
template <bool COUNT>
__device__ __forceinline__ uint32_t mc_h84_row(const McArgs &a, int64_t o, int64_t l, int64_t c4,
                                               uint32_t &type, uint32_t &xw, uint32_t (&cnt)[5]) {
  const int64_t i0 = (o * a.len + l) * a.inner + 4 * c4;
  xw = *reinterpret_cast<const uint32_t *>(a.x + i0);
  uint32_t f = 0, af = 0, n1 = 0, n2 = 0, data;
  const uint32_t cw = mc_noisy4<true, 8>(xw, (uint32_t)(a.offset0 + i0), a, f, af, 4);
  h84_decode4(cw, data, type, n1, n2);
  if (COUNT) {
    cnt[0] += f;
    cnt[1] += af;
    cnt[2] += n1;
    cnt[3] += n2;
  }
  return data;
}

__global__ __launch_bounds__(kBlock) void mc_h84_interp_kernel(McArgs a) {
  uint32_t c[5] = {0, 0, 0, 0, 0};
  const int64_t chunks = a.inner / 4;
  const int64_t strips = (a.len + kMcStrip - 1) / kMcStrip;
  const int64_t items = a.outer * strips * chunks;
  for (int64_t it = (int64_t)blockIdx.x * kBlock + threadIdx.x; it < items;
       it += (int64_t)gridDim.x * kBlock) {
    const int64_t c4 = it % chunks;
    const int64_t t = it / chunks;
    const int64_t sp = t % strips;
    const int64_t o = t / strips;
    const int64_t l0 = sp * kMcStrip, l1 = min<int64_t>(l0 + kMcStrip, a.len);
    // walk the strip with the previous / current / next decoded rows in registers
    uint32_t e_cur, x_cur, e_nxt, x_nxt, prev = 0, none[5];
    uint32_t cur = mc_h84_row<true>(a, o, l0, c4, e_cur, x_cur, c);
    for (int64_t l = l0; l < l1; ++l) {
      uint32_t nxt = cur;
      if (l + 1 < l1) nxt = mc_h84_row<true>(a, o, l + 1, c4, e_nxt, x_nxt, c);
      uint32_t out = sat15(cur);
      if (is_double(e_cur)) {  // the neighbours only matter here; past the strip, recompute
        // at most one neighbour lies outside the strip (strips hold >= 2 rows
        // unless the sequence has one position): one recompute site
        const bool out_l = l == l0 && l > 0, out_r = l + 1 == l1 && l + 1 < a.len;
        uint32_t ext = cur;
        if (out_l || out_r) {
          uint32_t tt, xx;
          ext = mc_h84_row<false>(a, o, out_l ? l - 1 : l + 1, c4, tt, xx, none);
        }
        const uint32_t left = l == 0 ? cur : (out_l ? ext : prev);
        const uint32_t right = l + 1 >= a.len ? cur : (out_r && !out_l ? ext : nxt);
        out = interp_word(cur, left, right, e_cur);
      }
      c[4] += mc_ne_bytes(out ^ x_cur);
      prev = cur;
      cur = nxt;
      e_cur = e_nxt;
      x_cur = x_nxt;
    }
  }
  flush_stats_n<5>(a.stats, c);
}

// Golay(24,12) trial over per-head rows: 4 codewords per lane; the tables live
// in LDS as in golay.hip
__global__ __launch_bounds__(kBlock) void mc_golay_kernel(McArgs a, const uint16_t *__restrict__ par,
                                                          const uint16_t *__restrict__ cor) {
  __shared__ __attribute__((aligned(16))) uint16_t lds[8192];
  {
    const u32x4 *p = reinterpret_cast<const u32x4 *>(par), *q = reinterpret_cast<const u32x4 *>(cor);
    u32x4 *l = reinterpret_cast<u32x4 *>(lds);
    for (int i = threadIdx.x; i < 512; i += kBlock) {
      l[i] = p[i];
      l[512 + i] = q[i];
    }
    __syncthreads();
  }
  uint32_t c[5] = {0, 0, 0, 0, 0};
  const int64_t m = a.outer * a.len * (a.inner / a.head_dim) * a.g;
  const int64_t groups = (m + 3) / 4;
  const uint32_t d = (uint32_t)a.head_dim, gg = (uint32_t)a.g;
  for (int64_t gi = (int64_t)blockIdx.x * kBlock + threadIdx.x; gi < groups;
       gi += (int64_t)gridDim.x * kBlock) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int64_t i = gi * 4 + k;
      if (i >= m) break;
      const int64_t row = i / gg;
      const uint32_t j = (uint32_t)(i - row * gg);
      const uint8_t *xr = a.x + row * d;
      const uint32_t v0 = xr[3 * j];
      const uint32_t v1 = 3 * j + 1 < d ? xr[3 * j + 1] : 0u;
      const uint32_t v2 = 3 * j + 2 < d ? xr[3 * j + 2] : 0u;
      const uint32_t dw = golay_pack(v0, v1, v2);
      const uint32_t g = (uint32_t)(a.offset0 + i);
      const uint32_t mk = philox_flip_mask<24>(a.seedmul + g * 24u, g, a.thr, 24);
      c[0] += __builtin_popcount(mk);
      c[1] += mk != 0;
      uint32_t cnt;
      const uint32_t dec = golay_decode1((dw | (uint32_t)lds[dw] << 12) ^ mk, lds, lds + 4096, cnt);
      c[2] += cnt & 3u;
      c[3] += cnt >> 2;
      const uint32_t diff = dec ^ dw;  // padding nibbles are 0 in dw; count the real ones only
      const uint32_t mask = 3 * j + 2 < d ? 0xFFFu : (3 * j + 1 < d ? 0xFFu : 0xFu);
      c[4] += ((diff & mask & 0xFu) != 0) + ((diff & mask & 0xF0u) != 0) + ((diff & mask & 0xF00u) != 0);
    }
  }
  flush_stats_n<5>(a.stats, c);
}

// dst[b * stride + w] += sum over the slots of buffer b, then zero the buffer
__global__ __launch_bounds__(kBlock) void stats_fold_kernel(uint64_t *stats, int64_t nbuf, int nwords,
                                                            int64_t *dst, int64_t stride) {
  const int64_t b = blockIdx.x;
  if (b >= nbuf) return;
  uint64_t *buf = stats + b * KVECC_STATS_WORDS;
  const int w = threadIdx.x;
  if (w < nwords) {
    unsigned long long sum = 0;
    for (int s = 0; s < KVECC_STATS_SLOTS; ++s) sum += buf[s * KVECC_STATS_STRIDE + w];
    dst[b * stride + w] += (int64_t)sum;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < KVECC_STATS_WORDS; i += kBlock) buf[i] = 0;
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_mc_trial(const uint8_t *x, int64_t outer, int64_t len, int64_t heads,
                             int64_t head_dim, int codec, float ber, int64_t seed, int64_t global_n,
                             int64_t offset0, uint64_t *stats, void *stream) {
  if (outer < 0 || len < 0 || heads < 0 || head_dim < 1 || global_n < 0 || offset0 < 0)
    return set_error(KVECC_EINVAL, "mc_trial: negative size/offset");
  if (!stats) return set_error(KVECC_EINVAL, "mc_trial: null stats");
  McArgs a;
  a.x = x;
  a.outer = outer;
  a.len = len;
  a.inner = heads * head_dim;
  a.head_dim = head_dim;
  a.g = (head_dim + 2) / 3;
  a.offset0 = offset0;
  a.thr = kvecc_ber_threshold(ber);
  a.stats = stats;
  const int64_t rows = outer * len * heads;
  const int64_t units = codec == KVECC_MC_GOLAY ? rows * a.g : rows * head_dim;
  if (units == 0) return KVECC_OK;
  if (!x) return set_error(KVECC_EINVAL, "mc_trial: null x");
  if (offset0 + units > global_n)
    return set_error(KVECC_EINVAL, "mc_trial: shard [%lld,%lld) exceeds global_n %lld", (long long)offset0,
                     (long long)(offset0 + units), (long long)global_n);
  hipStream_t st = as_stream(stream);
  switch (codec) {
    case KVECC_MC_H74:
    case KVECC_MC_H84:
    case KVECC_MC_H84_INTERP: {
      if (!aligned(x, 4)) return set_error(KVECC_EINVAL, "mc_trial: x must be 4-byte aligned");
      const int nb = codec == KVECC_MC_H74 ? 7 : 8;
      a.nbits = (uint32_t)nb;
      a.seedmul = (uint32_t)((uint64_t)seed * (uint64_t)((uint64_t)global_n * (uint64_t)nb));
      if (codec == KVECC_MC_H84_INTERP) {
        if (a.inner % 4) return set_error(KVECC_EINVAL, "mc_trial: interpolation needs heads*head_dim %% 4 == 0");
        const int64_t items = outer * ((len + kMcStrip - 1) / kMcStrip) * (a.inner / 4);
        KVECC_LAUNCH(mc_h84_interp_kernel, dim3(grid_for(items, kBlock, kMcPerCu)), dim3(kBlock), 0, st, a);
      } else if (codec == KVECC_MC_H84) {
        KVECC_LAUNCH((mc_hamming_kernel<true, 8>), dim3(grid_for((units + 3) / 4, kBlock, kMcPerCu)),
                     dim3(kBlock), 0, st, a);
      } else {
        KVECC_LAUNCH((mc_hamming_kernel<false, 7>), dim3(grid_for((units + 3) / 4, kBlock, kMcPerCu)),
                     dim3(kBlock), 0, st, a);
      }
      break;
    }
    case KVECC_MC_GOLAY: {
      a.nbits = 24;
      a.seedmul = (uint32_t)((uint64_t)seed * (uint64_t)((uint64_t)global_n * 24u));
      const uint16_t *par = golay_parity_table_dev(), *cor = golay_correct_table_dev();
      if (!par || !cor) return KVECC_EHIP;
      KVECC_LAUNCH(mc_golay_kernel, dim3(grid_for((units + 3) / 4, kBlock, kMcPerCu)), dim3(kBlock), 0, st, a,
                   par, cor);
      break;
    }
    default:
      return set_error(KVECC_EINVAL, "mc_trial: unknown codec %d", codec);
  }
  return check_launch("mc_trial");
}

KVECC_API int kvecc_stats_fold(uint64_t *stats, int64_t nbuf, int nwords, int64_t *dst, int64_t dst_stride,
                               void *stream) {
  if (nbuf < 0 || nwords < 0 || nwords > KVECC_STATS_STRIDE)
    return set_error(KVECC_EINVAL, "stats_fold: bad nbuf %lld / nwords %d", (long long)nbuf, nwords);
  if (nbuf == 0) return KVECC_OK;
  if (!stats || !dst) return set_error(KVECC_EINVAL, "stats_fold: null pointer");
  if (nbuf > 0x7FFFFFFF) return set_error(KVECC_EINVAL, "stats_fold: too many buffers");
  KVECC_LAUNCH(stats_fold_kernel, dim3((unsigned)nbuf), dim3(kBlock), 0, as_stream(stream), stats, nbuf, nwords,
               dst, dst_stride);
  return check_launch("stats_fold");
}

}  // extern "C"
