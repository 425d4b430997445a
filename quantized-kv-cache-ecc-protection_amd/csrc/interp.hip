// interp.hip -- temporal interpolation of SECDED double-error positions.
//
// Reference: ecc_codecs/triton_kernels/interpolation_triton.py:120-159 (kernel)
// and :162-265 (wrapper).  The kernel computes, in fp32,
//   r   = err == 2 ? (q[l-1] + q[l+1]) * 0.5 : q[l]      (clamped neighbours)
//   out = uint8(max(0, min(15, r + 0.5)))
// With 8-bit integer inputs every step is exact in fp32, so this equals the
// integer form  err == 2 ? min(15, (L + R + 1) >> 1) : min(15, q)  which the
// kernels evaluate SWAR on four bytes per register.
//
// gfx950 design: the tensor is addressed as [outer][len][inner] with the
// sequence axis in the middle, so any seq_dim is handled in place (the
// reference permutes + copies to make it the last axis).  When inner is a
// multiple of 16 each lane owns a 16-byte column chunk and walks kRows
// consecutive sequence positions, so every q row is loaded once per lane
// (plus a one-row halo) with 16-byte loads.  The reference's no-double fast
// path (:199-201: return q.clone() when no err == 2) is resolved without a host
// sync and without a separate scan of err: kvecc_interpolate_auto writes the
// interpolated (clamped) result in one pass while recording whether any double
// and any q > 15 was seen; the two differ only when there is no double and some
// q > 15, which a trailing copy kernel (a no-op otherwise) then handles.
#include "kvecc_internal.h"

namespace kvecc {

constexpr int kRows = 4;                       // positions per wave of a tile
constexpr int kTileWavesI = 8;                  // waves per workgroup tile
constexpr int kTileRows = kRows * kTileWavesI;  // 32 positions per tile
constexpr int kTileThreads = kTileWavesI * kWave;

// sat15 / avg_up / is_double / interp_word (four bytes per word): codec_math.h
__device__ __forceinline__ u32x4 interp_vec(u32x4 q, u32x4 l, u32x4 r, u32x4 e) {
  u32x4 o;
  o.x = interp_word(q.x, l.x, r.x, e.x);
  o.y = interp_word(q.y, l.y, r.y, e.y);
  o.z = interp_word(q.z, l.z, r.z, e.z);
  o.w = interp_word(q.w, l.w, r.w, e.w);
  return o;
}

// any byte of the word == 2 / > 15
__device__ __forceinline__ uint32_t seen_double(u32x4 e) {
  return is_double(e.x) | is_double(e.y) | is_double(e.z) | is_double(e.w);
}
__device__ __forceinline__ uint32_t seen_over15(u32x4 q) {
  return (q.x | q.y | q.z | q.w) & 0xF0F0F0F0u;
}

// vector path (inner % 16 == 0): workgroup tiles of 64 column chunks (1 KiB)
// x kTileRows positions.  Wave w owns positions [w kRows, w kRows + kRows) of
// the tile and loads its q and err rows once, non-temporally; it publishes its
// first and last q row in LDS and takes its neighbour waves' edge rows from
// there after one barrier, so only the tile's two outer halo rows come from
// HBM: 2 / 32 of q re-read instead of the 2 / 8 of the round-1 per-lane row
// blocks (63.5 against 68.9 us at [8,4096,32,128], tools/exp/run_r05.py,
// profiles/r05/exp_r05.log).  Ragged shapes: lanes past the last chunk and
// rows past the sequence end load and store nothing; the clamped neighbours
// (q[max(l-1,0)], q[min(l+1,len-1)]) come from the same rows.
// RECORD: no gate; flags[0] = epoch if any err == 2, flags[1] = epoch if any
// q > 15, one store per wave that saw one and found the word not yet stamped
// (no barrier after the stores, no zeroing pass)
template <bool RECORD>
__global__ __launch_bounds__(kTileThreads) void interp_tile_kernel(const u32x4 *__restrict__ q,
                                                                  const u32x4 *__restrict__ err,
                                                                  u32x4 *__restrict__ out, int64_t len,
                                                                  int64_t chunks,
                                                                  const int32_t *__restrict__ gate,
                                                                  int32_t *__restrict__ flags, int32_t epoch) {
  __shared__ u32x4 edge[2][kTileWavesI][kWave];  // [first, last row][wave][lane]
  const bool pass = !RECORD && gate != nullptr && *gate == 0;
  const int lane = threadIdx.x & (kWave - 1);
  const int w = threadIdx.x / kWave;
  const int64_t cgroups = (chunks + kWave - 1) / kWave;
  const int64_t rtiles = (len + kTileRows - 1) / kTileRows;
  const int64_t t = blockIdx.x;
  const int64_t cg = t % cgroups;
  const int64_t rt = (t / cgroups) % rtiles;
  const int64_t o = t / (cgroups * rtiles);
  const int64_t c = cg * kWave + lane;
  const bool col = c < chunks;
  const int64_t l0 = rt * kTileRows + (int64_t)w * kRows;
  const int nrow = (int)max<int64_t>(0, min<int64_t>(kRows, len - l0));  // wave-uniform
  const int64_t base = o * len * chunks + c;
  u32x4 qr[kRows + 2], er[kRows];
#pragma unroll
  for (int k = 0; k < kRows; ++k)
    if (k < nrow && col) qr[k + 1] = ld_stream(q + base + (l0 + k) * chunks);
  // the tile's outer neighbours: the row above the first wave, the row below
  // the wave holding the tile's (or the sequence's) last row -- issued before
  // the err rows, so the edge waves' halo is not queued behind them
  const bool top = w == 0 && l0 > 0;
  const bool last = nrow > 0 && (w == kTileWavesI - 1 || l0 + kRows >= len);
  const bool bottom = last && l0 + nrow < len;
  if (!pass && col && top) qr[0] = ld_stream(q + base + (l0 - 1) * chunks);
  if (!pass && col && bottom) qr[kRows + 1] = ld_stream(q + base + (l0 + nrow) * chunks);
  if (!pass) {
#pragma unroll
    for (int k = 0; k < kRows; ++k)
      if (k < nrow && col) er[k] = ld_stream(err + base + (l0 + k) * chunks);
  }
  if (!pass) {
    if (nrow > 0) {
      edge[0][w][lane] = qr[1];
      edge[1][w][lane] = qr[kRows];  // (a partial wave is the tile's last: never read)
    }
    __syncthreads();
    if (nrow > 0 && col) {
      if (l0 == 0) qr[0] = qr[1];                  // q[max(l-1, 0)]
      else if (w > 0) qr[0] = edge[1][w - 1][lane];
      if (!last) qr[kRows + 1] = edge[0][w + 1][lane];
      else if (!bottom) qr[nrow + 1] = qr[nrow];   // q[min(l+1, len-1)]
      else if (nrow < kRows) qr[nrow + 1] = qr[kRows + 1];
    }
  }
  uint32_t dbl = 0, over = 0;
#pragma unroll
  for (int k = 0; k < kRows; ++k) {
    if (k >= nrow || !col) break;
    const u32x4 v = pass ? qr[k + 1] : interp_vec(qr[k + 1], qr[k], qr[k + 2], er[k]);
    st_stream(out + base + (l0 + k) * chunks, v);
    if (RECORD) {
      dbl |= seen_double(er[k]);
      over |= seen_over15(qr[k + 1]);
    }
  }
  if (RECORD) {
    const bool d = __any(dbl != 0), ov = __any(over != 0);
    if (lane == 0) {
      if (d && __builtin_nontemporal_load(flags) != epoch) flags[0] = epoch;
      if (ov && __builtin_nontemporal_load(flags + 1) != epoch) flags[1] = epoch;
    }
  }
}

// (Strips -- a lane walking 16-128 rows of its column chunk and carrying the
// last two q rows from block to block, so the halo costs 2/strip instead of
// 2/8 -- took 80.4-83.4 us against 76.8 for the row blocks above: the longer
// dependent chain per lane costs more than the 12.5 % of re-fetched bytes, most
// of which hit L2; profiles/r02/interp_strips.log.)

// scalar path: one element per lane
template <bool RECORD>
__global__ __launch_bounds__(kBlock) void interp_scalar_kernel(const uint8_t *__restrict__ q,
                                                               const uint8_t *__restrict__ err,
                                                               uint8_t *__restrict__ out,
                                                               int64_t outer, int64_t len,
                                                               int64_t inner,
                                                               const int32_t *__restrict__ gate,
                                                               int32_t *__restrict__ flags,
                                                               int32_t epoch) {
  const bool pass = !RECORD && gate != nullptr && *gate == 0;
  bool dbl = false, over = false;
  const int64_t total = outer * len * inner;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * kBlock) {
    if (pass) {
      out[i] = q[i];
      continue;
    }
    const int64_t c = i % inner;
    const int64_t l = (i / inner) % len;
    const int64_t rowbase = i - l * inner;
    const uint32_t left = q[rowbase + (l > 0 ? l - 1 : 0) * inner];
    const uint32_t right = q[rowbase + (l + 1 < len ? l + 1 : len - 1) * inner];
    (void)c;
    out[i] = (uint8_t)interp_word(q[i], left, right, err[i]);
    if (RECORD) {
      dbl |= err[i] == 2;
      over |= q[i] > 15;
    }
  }
  if (RECORD) {
    const bool d = __syncthreads_or(dbl), o = __syncthreads_or(over);
    if (threadIdx.x == 0) {
      if (d) flags[0] = epoch;
      if (o) flags[1] = epoch;
    }
  }
}

// after a RECORD pass: no double anywhere but some q > 15 -> out = q (the
// reference returns an unclamped clone); otherwise every workgroup exits at
// once.  A small grid: the copy is the rare branch, the exit is the common one.
__global__ __launch_bounds__(kBlock) void interp_fixup_kernel(const uint8_t *__restrict__ q,
                                                              uint8_t *__restrict__ out, int64_t n,
                                                              const int32_t *__restrict__ flags,
                                                              int32_t epoch, bool vec) {
  if (flags[0] == epoch || flags[1] != epoch) return;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  const int64_t tid = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  int64_t done = 0;
  if (vec) {
    const int64_t nv = n / 16;
    for (int64_t i = tid; i < nv; i += stride)
      reinterpret_cast<u32x4 *>(out)[i] = reinterpret_cast<const u32x4 *>(q)[i];
    done = nv * 16;
  }
  for (int64_t i = done + tid; i < n; i += stride) out[i] = q[i];
}

__device__ __forceinline__ bool has_byte(u32x4 v, uint32_t pat) {
  const uint32_t w[4] = {v.x ^ pat, v.y ^ pat, v.z ^ pat, v.w ^ pat};
  bool hit = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) hit |= ((w[k] - 0x01010101u) & ~w[k] & 0x80808080u) != 0;  // a zero byte
  return hit;
}

// four 16-byte non-temporal loads in flight per lane
__global__ __launch_bounds__(kBlock) void any_equal_kernel(const uint8_t *__restrict__ x, int64_t n,
                                                           uint32_t value, int32_t *__restrict__ flag) {
  constexpr int kU = 4;
  bool hit = false;
  const int64_t nvec = (reinterpret_cast<uintptr_t>(x) % 16 == 0) ? n / 16 : 0;
  const u32x4 *xv = reinterpret_cast<const u32x4 *>(x);
  const uint32_t pat = value * 0x01010101u;
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  for (; i + (kU - 1) * stride < nvec; i += kU * stride) {
    u32x4 v[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) v[u] = ld_stream(xv + i + u * stride);
#pragma unroll
    for (int u = 0; u < kU; ++u) hit |= has_byte(v[u], pat);
  }
  for (; i < nvec; i += stride) hit |= has_byte(ld_stream(xv + i), pat);
  for (int64_t j = nvec * 16 + (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += stride)
    hit |= x[j] == value;
  // one plain store per hitting workgroup: thousands of same-address atomics
  // serialise at ~10 ns each (they cost more than the scan)
  if (__syncthreads_or(hit) && threadIdx.x == 0) *flag = 1;
}

// bytes of a that differ from b: four 16-byte non-temporal loads of each in
// flight per lane; per word, the nonzero bytes of a ^ b are folded to bit 0 of
// each byte and counted with one popcount
__device__ __forceinline__ uint32_t ne_bytes(uint32_t x) {
  x |= x >> 4;
  x |= x >> 2;
  x |= x >> 1;
  return __builtin_popcount(x & 0x01010101u);
}

__global__ __launch_bounds__(kBlock) void count_ne_kernel(const uint8_t *__restrict__ a,
                                                          const uint8_t *__restrict__ b, int64_t n,
                                                          uint64_t *__restrict__ stats) {
  constexpr int kU = 4;
  uint32_t cnt = 0;
  const bool vec = (reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) % 16 == 0;
  const int64_t nvec = vec ? n / 16 : 0;
  const u32x4 *av = reinterpret_cast<const u32x4 *>(a), *bv = reinterpret_cast<const u32x4 *>(b);
  const int64_t stride = (int64_t)gridDim.x * kBlock;
  int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
  for (; i + (kU - 1) * stride < nvec; i += kU * stride) {
    u32x4 x[kU], y[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      x[u] = ld_stream(av + i + u * stride);
      y[u] = ld_stream(bv + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < kU; ++u)
      cnt += ne_bytes(x[u].x ^ y[u].x) + ne_bytes(x[u].y ^ y[u].y) + ne_bytes(x[u].z ^ y[u].z) +
             ne_bytes(x[u].w ^ y[u].w);
  }
  for (; i < nvec; i += stride) {
    const u32x4 x = ld_stream(av + i), y = ld_stream(bv + i);
    cnt += ne_bytes(x.x ^ y.x) + ne_bytes(x.y ^ y.y) + ne_bytes(x.z ^ y.z) + ne_bytes(x.w ^ y.w);
  }
  for (int64_t j = nvec * 16 + (int64_t)blockIdx.x * kBlock + threadIdx.x; j < n; j += stride)
    cnt += a[j] != b[j];
  flush_stats2(stats, cnt, 0u);
}

template <bool RECORD>
static void launch_interp(const uint8_t *q, const uint8_t *err, uint8_t *out, int64_t outer,
                          int64_t len, int64_t inner, const int32_t *gate, int32_t *flags,
                          int32_t epoch, hipStream_t st) {
  if (inner % 16 == 0 && aligned(q, 16) && aligned(err, 16) && aligned(out, 16)) {
    const int64_t chunks = inner / 16;
    const int64_t tiles = outer * ((len + kTileRows - 1) / kTileRows) * ((chunks + kWave - 1) / kWave);
    KVECC_LAUNCH((interp_tile_kernel<RECORD>), dim3((unsigned)tiles), dim3(kTileThreads), 0, st,
                 reinterpret_cast<const u32x4 *>(q), reinterpret_cast<const u32x4 *>(err),
                 reinterpret_cast<u32x4 *>(out), len, chunks, gate, flags, epoch);
  } else {
    KVECC_LAUNCH((interp_scalar_kernel<RECORD>), dim3(grid_for(outer * len * inner, kBlock)),
                 dim3(kBlock), 0, st, q, err, out, outer, len, inner, gate, flags, epoch);
  }
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int kvecc_interpolate(const uint8_t *q, const uint8_t *err, uint8_t *out,
                                int64_t outer, int64_t len, int64_t inner, const int32_t *gate,
                                void *stream) {
  if (outer < 0 || len < 0 || inner < 0) return set_error(KVECC_EINVAL, "interpolate: negative size");
  const int64_t total = outer * len * inner;
  if (total == 0) return KVECC_OK;
  if (!q || !err || !out) return set_error(KVECC_EINVAL, "interpolate: null pointer");
  launch_interp<false>(q, err, out, outer, len, inner, gate, nullptr, 0, as_stream(stream));
  return check_launch("interpolate");
}

KVECC_API int kvecc_interpolate_auto(const uint8_t *q, const uint8_t *err, uint8_t *out,
                                     int64_t outer, int64_t len, int64_t inner, int32_t *flags,
                                     int32_t epoch, void *stream) {
  if (outer < 0 || len < 0 || inner < 0)
    return set_error(KVECC_EINVAL, "interpolate_auto: negative size");
  if (!flags) return set_error(KVECC_EINVAL, "interpolate_auto: null flags");
  if (epoch == 0) return set_error(KVECC_EINVAL, "interpolate_auto: epoch must be non-zero");
  const int64_t total = outer * len * inner;
  if (total == 0) return KVECC_OK;
  if (!q || !err || !out) return set_error(KVECC_EINVAL, "interpolate_auto: null pointer");
  hipStream_t st = as_stream(stream);
  launch_interp<true>(q, err, out, outer, len, inner, nullptr, flags, epoch, st);
  KVECC_LAUNCH(interp_fixup_kernel, dim3(64), dim3(kBlock), 0, st, q, out, total, flags, epoch,
               aligned(q, 16) && aligned(out, 16));
  return check_launch("interpolate_auto");
}

KVECC_API int kvecc_count_ne_u8(const uint8_t *a, const uint8_t *b, int64_t n, uint64_t *stats,
                                void *stream) {
  if (n < 0) return set_error(KVECC_EINVAL, "count_ne_u8: negative n");
  if (n == 0) return KVECC_OK;
  if (!a || !b || !stats) return set_error(KVECC_EINVAL, "count_ne_u8: null pointer");
  KVECC_LAUNCH(count_ne_kernel, dim3(grid_for(n, (int64_t)kBlock * 64, 8)), dim3(kBlock), 0,
               as_stream(stream), a, b, n, stats);
  return check_launch("count_ne_u8");
}

KVECC_API int kvecc_any_equal_u8(const uint8_t *x, int64_t n, uint8_t value, int32_t *flag,
                                 void *stream) {
  if (n < 0) return set_error(KVECC_EINVAL, "any_equal_u8: negative n");
  if (!flag) return set_error(KVECC_EINVAL, "any_equal_u8: null flag");
  hipStream_t st = as_stream(stream);
  hipError_t e = hipMemsetAsync(flag, 0, sizeof(int32_t), st);
  if (e != hipSuccess) return set_error(KVECC_EHIP, "any_equal_u8: %s", hipGetErrorString(e));
  if (n == 0) return KVECC_OK;
  if (!x) return set_error(KVECC_EINVAL, "any_equal_u8: null input");
  KVECC_LAUNCH(any_equal_kernel, dim3(grid_for(n, (int64_t)kBlock * 64, 8)), dim3(kBlock), 0,
                     st, x, n, (uint32_t)value, flag);
  return check_launch("any_equal_u8");
}

}  // extern "C"
