// hamming.hip -- Hamming(7,4) SEC and Hamming(8,4) SECDED encode/decode.
//
// Reference: ecc_codecs/triton_kernels/hamming74_triton.py:48-162 and
// hamming84_triton.py:50-209.  One codeword per byte, data in the low nibble,
// layout [d0 d1 d2 d3 p0 p1 p2 (overall parity)].
//
// gfx950 design: the op is HBM-bound (2-3 B per value), so every lane moves
// 16 B per non-temporal load/store (global_load_dwordx4), and the bit algebra
// runs SWAR on four codewords per 32-bit register instead of the reference's
// bit-by-bit extraction.  Per-byte syndromes come from masked byte parities;
// the 8-entry syndrome->position table of config.py:131-161 is folded into
// closed-form flip masks (only data-bit flips matter for the output).
// Statistics are reduced per workgroup into the sharded counters (kvecc.h).
#include "kvecc_internal.h"

namespace kvecc {

// Geometry from interleaved cold-cache A/B runs (tools/exp/run_ham.py): one
// 16-B vector per lane per tile and up to 64 workgroups per CU beat 2-4
// vectors per lane by 6-8% (encode 5.9 TB/s, decode 5.7 TB/s on MI355X).
constexpr int kUnroll = 1;   // 16-B vectors per lane per tile
constexpr int kPerCu = 64;   // workgroups per CU before grid-striding

// encoders and decoders: codec_math.h (shared with the host backend)
struct H74Enc {
  __device__ __forceinline__ static uint32_t op(uint32_t w) { return h74_encode4(w); }
};
struct H84Enc {
  __device__ __forceinline__ static uint32_t op(uint32_t w) { return h84_encode4(w); }
};

template <class Op>
__global__ __launch_bounds__(kBlock) void encode_kernel(const u32x4 *__restrict__ in,
                                                        u32x4 *__restrict__ out, int64_t nvec) {
  const int64_t tile = (int64_t)kBlock * kUnroll;
  for (int64_t base = (int64_t)blockIdx.x * tile; base < nvec; base += (int64_t)gridDim.x * tile) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      int64_t i = base + u * kBlock + threadIdx.x;
      if (i < nvec) v[u] = ld_stream(in + i);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      int64_t i = base + u * kBlock + threadIdx.x;
      if (i < nvec) {
        u32x4 r;
        r.x = Op::op(v[u].x);
        r.y = Op::op(v[u].y);
        r.z = Op::op(v[u].z);
        r.w = Op::op(v[u].w);
        st_stream(out + i, r);
      }
    }
  }
}

template <class Op>
__global__ __launch_bounds__(kBlock) void encode_bytes_kernel(const uint8_t *__restrict__ in,
                                                              uint8_t *__restrict__ out,
                                                              int64_t begin, int64_t n) {
  for (int64_t i = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock)
    out[i] = (uint8_t)Op::op(in[i]);
}

__device__ __forceinline__ void dec84_word(uint32_t w, uint32_t &data, uint32_t &type,
                                           uint32_t &n_single, uint32_t &n_double) {
  h84_decode4(w, data, type, n_single, n_double);
}
__device__ __forceinline__ void dec74_word(uint32_t w, uint32_t &data, uint32_t &flag,
                                           uint32_t &n_flag) {
  h74_decode4(w, data, flag, n_flag);
}

template <bool H84, bool WITH_AUX, bool WITH_STATS>
__global__ __launch_bounds__(kBlock) void decode_kernel(const u32x4 *__restrict__ cw,
                                                        u32x4 *__restrict__ data,
                                                        u32x4 *__restrict__ aux, int64_t nvec,
                                                        uint64_t *__restrict__ stats) {
  const int64_t tile = (int64_t)kBlock * kUnroll;
  uint32_t c0 = 0, c1 = 0;
  for (int64_t base = (int64_t)blockIdx.x * tile; base < nvec; base += (int64_t)gridDim.x * tile) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      int64_t i = base + u * kBlock + threadIdx.x;
      if (i < nvec) v[u] = ld_stream(cw + i);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      int64_t i = base + u * kBlock + threadIdx.x;
      if (i < nvec) {
        const uint32_t w[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
        uint32_t dd[4], tt[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          if (H84)
            dec84_word(w[k], dd[k], tt[k], c0, c1);
          else
            dec74_word(w[k], dd[k], tt[k], c0);
        }
        u32x4 d, t;
        d.x = dd[0]; d.y = dd[1]; d.z = dd[2]; d.w = dd[3];
        t.x = tt[0]; t.y = tt[1]; t.z = tt[2]; t.w = tt[3];
        st_stream(data + i, d);
        if (WITH_AUX) st_stream(aux + i, t);
      }
    }
  }
  if (WITH_STATS) flush_stats2(stats, c0, c1);
}

template <bool H84>
__global__ __launch_bounds__(kBlock) void decode_bytes_kernel(const uint8_t *__restrict__ cw,
                                                              uint8_t *__restrict__ data,
                                                              uint8_t *__restrict__ aux,
                                                              int64_t begin, int64_t n,
                                                              uint64_t *__restrict__ stats) {
  uint32_t c0 = 0, c1 = 0;
  for (int64_t i = begin + (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    uint32_t d, t;
    if (H84)
      dec84_word(cw[i], d, t, c0, c1);
    else
      dec74_word(cw[i], d, t, c0);
    data[i] = (uint8_t)d;
    if (aux) aux[i] = (uint8_t)t;
  }
  if (stats) flush_stats2(stats, c0, c1);
}

template <class Op>
static int launch_encode(const uint8_t *in, uint8_t *out, int64_t n, void *stream, const char *name) {
  if (n < 0) return set_error(KVECC_EINVAL, "%s: negative n", name);
  if (n == 0) return KVECC_OK;
  if (!in || !out) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (aligned(in, 16) && aligned(out, 16)) {
    int64_t nvec = n / 16;
    if (nvec > 0) {
      unsigned g = grid_for(nvec, (int64_t)kBlock * kUnroll, kPerCu);
      KVECC_LAUNCH(encode_kernel<Op>, dim3(g), dim3(kBlock), 0, st,
                         reinterpret_cast<const u32x4 *>(in), reinterpret_cast<u32x4 *>(out), nvec);
    }
    done = nvec * 16;
  }
  if (done < n) {
    unsigned g = grid_for(n - done, kBlock);
    KVECC_LAUNCH(encode_bytes_kernel<Op>, dim3(g), dim3(kBlock), 0, st, in, out, done, n);
  }
  return check_launch(name);
}

template <bool H84>
static int launch_decode(const uint8_t *cw, uint8_t *data, uint8_t *aux, int64_t n,
                         uint64_t *stats, void *stream, const char *name) {
  if (n < 0) return set_error(KVECC_EINVAL, "%s: negative n", name);
  if (n == 0) return KVECC_OK;
  if (!cw || !data) return set_error(KVECC_EINVAL, "%s: null pointer", name);
  hipStream_t st = as_stream(stream);
  int64_t done = 0;
  if (aligned(cw, 16) && aligned(data, 16) && (!aux || aligned(aux, 16))) {
    int64_t nvec = n / 16;
    if (nvec > 0) {
      unsigned g = grid_for(nvec, (int64_t)kBlock * kUnroll, kPerCu);
      auto c = reinterpret_cast<const u32x4 *>(cw);
      auto d = reinterpret_cast<u32x4 *>(data);
      auto a = reinterpret_cast<u32x4 *>(aux);
      if (aux && stats)
        KVECC_LAUNCH((decode_kernel<H84, true, true>), dim3(g), dim3(kBlock), 0, st, c, d, a, nvec, stats);
      else if (aux)
        KVECC_LAUNCH((decode_kernel<H84, true, false>), dim3(g), dim3(kBlock), 0, st, c, d, a, nvec, stats);
      else if (stats)
        KVECC_LAUNCH((decode_kernel<H84, false, true>), dim3(g), dim3(kBlock), 0, st, c, d, a, nvec, stats);
      else
        KVECC_LAUNCH((decode_kernel<H84, false, false>), dim3(g), dim3(kBlock), 0, st, c, d, a, nvec, stats);
    }
    done = nvec * 16;
  }
  if (done < n) {
    unsigned g = grid_for(n - done, kBlock);
    KVECC_LAUNCH(decode_bytes_kernel<H84>, dim3(g), dim3(kBlock), 0, st, cw, data, aux, done, n, stats);
  }
  return check_launch(name);
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_hamming74_encode(const uint8_t *in, uint8_t *out, int64_t n, void *stream) {
  return launch_encode<H74Enc>(in, out, n, stream, "hamming74_encode");
}

KVECC_API int kvecc_hamming84_encode(const uint8_t *in, uint8_t *out, int64_t n, void *stream) {
  return launch_encode<H84Enc>(in, out, n, stream, "hamming84_encode");
}

KVECC_API int kvecc_hamming74_decode(const uint8_t *cw, uint8_t *data, uint8_t *flag, int64_t n,
                                     uint64_t *stats, void *stream) {
  return launch_decode<false>(cw, data, flag, n, stats, stream, "hamming74_decode");
}

KVECC_API int kvecc_hamming84_decode(const uint8_t *cw, uint8_t *data, uint8_t *error_type,
                                     int64_t n, uint64_t *stats, void *stream) {
  return launch_decode<true>(cw, data, error_type, n, stats, stream, "hamming84_decode");
}

}  // extern "C"
