// kvecc_internal.h -- shared device/host helpers for the gfx950 codec kernels.
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <type_traits>
#include <stdint.h>

#include "codec_math.h"
#include "kvecc.h"

namespace kvecc {

// ---- vector types -----------------------------------------------------------
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;
constexpr int kBlock = 256;  // 4 waves

// ---- error state (runtime.hip) --------------------------------------------
int set_error(int code, const char *fmt, ...);
int check_launch(const char *what);
int cu_count();               // CUs of the current device (cached)
int current_device();
// Golay tables on the current device (uploaded on first use):
//   parity[d]   (uint16) = 12 parity bits of data word d       (encode, syndrome)
//   correct[s]  (uint16) = data-error(12) | count(3) << 12      (decode)
const uint16_t *golay_parity_table_dev();
const uint16_t *golay_correct_table_dev();
// Golay tables for paged attention (uint32[8192]): data nibbles spread one per
// byte, spread(x) = x&15 | (x>>4&15)<<8 | (x>>8&15)<<16, so a value converts
// with one v_cvt_f32_ubyteN:
//   [0, 4096)    spread(d) | parity(d) << 20
//   [4096, 8192) spread(data error of syndrome s) | ((count(s) & 3) | unc << 6) << 24
//                (count 0-3 bits corrected; uncorrectable: spread part 0, byte 3 = 0x40)
const uint32_t *golay_attn_table_dev();
// the attention split kernels' layout, for words holding codeword << 2: data
// nibbles at bits 0-3, 8-11, 28-31 and parity(d) << 14 (where such a word holds
// the received parity); correction half without the count byte (syndrome
// offset = ((w ^ P) & 0x3FFC000) >> 12)
const uint32_t *golay_attn_x_table_dev();
// packed decode tables, 24 KiB: uint16 [4096] parity(lo) << 2, then uint32
// [4096] error data | (bits corrected & 3) << 24 | uncorrectable << 31
const uint8_t *golay_pk_table_dev();
// Counter slots of the dynamically scheduled kernels (runtime.hip
// counter_slot): zero at launch, owned by one launch until it exits, left zero
// (each counter's last user resets it).  Eager launches get one slot per
// stream, captured launches one per (capture, stream), so two launches that
// can overlap never share a slot.  A slot holds
//   [0, kDynSlotWords): the work counters of the tile kernels (shim.hip,
//     golay.hip, packed.hip; TileSchedule), kDynCounters counters kDynStride
//     words apart;
//   [kDynSlotWords, +kAttnCtrPerSlot): the split counters of the paged-attention
//     fused combine, one per (batch, head group).
constexpr int kDynCounters = 128;
constexpr int kDynStride = 64;  // uint32 words (256 B) between counters
constexpr int kDynSlotWords = kDynCounters * kDynStride;
constexpr int kAttnCtrPerSlot = 4096;
constexpr int kSlotWords = kDynSlotWords + kAttnCtrPerSlot;
uint32_t *counter_slot(void *stream);  // nullptr on error (kvecc_last_error set)
inline uint32_t *shim_dyn_slot(void *stream) { return counter_slot(stream); }
inline uint32_t *attn_counter_slot(void *stream) {
  uint32_t *s = counter_slot(stream);
  return s ? s + kDynSlotWords : nullptr;
}
// host-side table builders (product copy, independent of the test oracle)
void build_golay_parity_table(uint16_t *out4096);
void build_golay_correct_table(uint16_t *out4096);

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// ---- launch timing (kvecc_time_next_launch) -----------------------------------
// When armed, the next kernel launched by this thread carries the events in its
// own dispatch (hipExtLaunchKernel): start/end stamps with no marker packets
// between kernels.  Every launch site goes through KVECC_LAUNCH.
struct LaunchTiming {
  hipEvent_t start, stop;
};
extern thread_local LaunchTiming g_launch_timing;

#define KVECC_LAUNCH(KERNEL, GRID, BLOCK, SHMEM, STREAM, ...)                                 \
  do {                                                                                        \
    if (::kvecc::g_launch_timing.start || ::kvecc::g_launch_timing.stop) {                    \
      const ::kvecc::LaunchTiming t_ = ::kvecc::g_launch_timing;                              \
      ::kvecc::g_launch_timing = {nullptr, nullptr};                                          \
      hipExtLaunchKernelGGL(KERNEL, GRID, BLOCK, SHMEM, STREAM, t_.start, t_.stop, 0u, __VA_ARGS__); \
    } else {                                                                                  \
      hipLaunchKernelGGL(KERNEL, GRID, BLOCK, SHMEM, STREAM, __VA_ARGS__);                    \
    }                                                                                         \
  } while (0)

inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// grid for a grid-stride loop over `work` items of `per_block` each: enough
// blocks to fill the chip (8 per CU), never more than there is work.
inline unsigned grid_for(int64_t work, int64_t per_block, int per_cu = 8) {
  int64_t need = cdiv(work, per_block);
  int64_t cap = (int64_t)cu_count() * per_cu;
  if (need > cap) need = cap;
  if (need < 1) need = 1;
  return (unsigned)need;
}

inline bool aligned(const void *p, uintptr_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

// ---- device helpers ----------------------------------------------------------

// Phase boundary of a wave-private LDS tile (lanes exchange data through LDS
// with accesses of different vector types).  wave_barrier alone is only a
// scheduling/convergence hint; the wavefront-scope release/acquire fences make
// the LDS ordering a guarantee of the memory model instead of current codegen
// (they emit s_waitcnt lgkmcnt, no cache maintenance for LDS).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// a wave-uniform value the compiler cannot prove uniform (it came through a
// vector load): readfirstlane, so buffer descriptors built from it live in
// SGPRs instead of a waterfall loop around every buffer load
__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ const char *uni(const char *p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  return reinterpret_cast<const char *>((uint64_t)uni((uint32_t)v) | (uint64_t)uni((uint32_t)(v >> 32)) << 32);
}

// a wave-uniform load through the scalar cache (s_load: counted by lgkmcnt, so
// it does not wait behind the wave's outstanding vector stores like a vector load)
__device__ __forceinline__ int32_t ld_scalar(const int32_t *p) {
  return *(const __attribute__((address_space(4))) int32_t *)uni(reinterpret_cast<const char *>(p));
}

// dequantization (n - 8) * s, rounded to fp32 as its own operation.  Left to
// itself the compiler may contract the product with a following fp16/bf16
// conversion into v_fma_mix*_f16, which rounds the exact product once, while
// the reference (and the host twin) round to fp32 first: 1 ulp apart.
// (Neither __fmul_rn nor `#pragma clang fp contract(off)` stops that combine;
// an empty asm on the fp32 product does.)
__device__ __forceinline__ float dequant1(uint32_t n, float s) {
  float x = ((float)n - 8.0f) * s;
  asm volatile("" : "+v"(x));
  return x;
}

// ---- packed dequantization ----------------------------------------------------
// (n - 8) * s exactly as the reference computes it (fp32 subtract, fp32 product,
// then one RNE conversion), two values per instruction: per 8 values 8
// v_cvt_f32_ubyte, 4 v_pk_add_f32, 4 v_pk_mul_f32, 4 v_cvt_pk_{f16,bf16}_f32
// (dequant1 with scalar conversions took ~4.5 VALU ops per value, and its
// volatile asm turned a `dead ? 0 : ...` per value into a branch per value).
// A missing block's rows decode to n = 0 with scale 0 (their loads fall
// outside the buffer descriptors); `dead` makes them n = 8, so they give
// (8 - 8) * 0 = +0, where n = 0 would give -0.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

// 4 nibble bytes -> 4 fp32 values, as two pairs
__device__ __forceinline__ void dq4(uint32_t nb, float s, f32x2 &lo, f32x2 &hi) {
  const f32x2 ss = {s, s}, m8 = {-8.0f, -8.0f};
  const f32x2 a = {(float)(nb & 0xFFu), (float)(nb >> 8 & 0xFFu)};
  const f32x2 b = {(float)(nb >> 16 & 0xFFu), (float)(nb >> 24)};
  f32x2 x = a + m8, y = b + m8;
  asm("" : "+v"(x), "+v"(y));  // (n - 8) exactly, then the product: no fma contraction
  lo = x * ss;
  hi = y * ss;
  asm("" : "+v"(lo), "+v"(hi));  // rounded to fp32 here: no v_fma_mix with the conversion
}

template <typename TO>
__device__ __forceinline__ uint32_t pack2(f32x2 v) {
  if constexpr (std::is_same<TO, __half>::value)
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
  else
    return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}

// the 16 output bytes of VPL nibble bytes (fp16/bf16: nb[0..1], fp32: nb[0])
template <typename TO>
__device__ __forceinline__ u32x4 dq16(const uint32_t *nb, float s, bool dead) {
  const uint32_t d8 = dead ? 0x08080808u : 0u;
  f32x2 v[4];
  dq4(nb[0] | d8, s, v[0], v[1]);
  if constexpr (sizeof(TO) == 4) {
    return u32x4{__float_as_uint(v[0].x), __float_as_uint(v[0].y), __float_as_uint(v[1].x),
                 __float_as_uint(v[1].y)};
  } else {
    dq4(nb[1] | d8, s, v[2], v[3]);
    return u32x4{pack2<TO>(v[0]), pack2<TO>(v[1]), pack2<TO>(v[2]), pack2<TO>(v[3])};
  }
}

// element conversions of the fused kernels (fp32 / fp16 / bf16, RNE on the way out)
template <typename T>
__device__ __forceinline__ float to_f32(T v);
template <>
__device__ __forceinline__ float to_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ float to_f32<__half>(__half v) { return __half2float(v); }
template <>
__device__ __forceinline__ float to_f32<__hip_bfloat16>(__hip_bfloat16 v) {
  return __bfloat162float(v);
}

template <typename T>
__device__ __forceinline__ T from_f32(float v);
template <>
__device__ __forceinline__ float from_f32<float>(float v) { return v; }
template <>
__device__ __forceinline__ __half from_f32<__half>(float v) { return __float2half_rn(v); }
template <>
__device__ __forceinline__ __hip_bfloat16 from_f32<__hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}


// DPP move inside a 16-lane row (CTRL: quad_perm 0x00-0xFF, row_mirror 0x140,
// row_half_mirror 0x141); no LDS round trip, unlike __shfl_xor's ds_bpermute
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, true);
}

// max over each aligned group of G lanes (G a power of two <= 64) of
// NON-NEGATIVE floats, result in every lane of the group.  Non-negative floats
// order like their bit patterns, so this is an unsigned max, which lets the
// DPP move fold into v_max_u32 (no canonicalize).  DPP for the steps inside a
// row, ds_bpermute across rows.
template <int G>
__device__ __forceinline__ float group_max_nonneg(float v) {
  uint32_t u = __float_as_uint(v);
  if (G >= 2) u = max(u, dpp_u32<0xB1>(u));    // quad_perm [1,0,3,2]: lane ^ 1
  if (G >= 4) u = max(u, dpp_u32<0x4E>(u));    // quad_perm [2,3,0,1]: lane ^ 2
  if (G >= 8) u = max(u, dpp_u32<0x141>(u));   // row_half_mirror: quad 0 <-> quad 1
  if (G >= 16) u = max(u, dpp_u32<0x140>(u));  // row_mirror: half 0 <-> half 1
  if (G >= 32) u = max(u, (uint32_t)__shfl_xor((int)u, 16, kWave));
  if (G >= 64) u = max(u, (uint32_t)__shfl_xor((int)u, 32, kWave));
  return __uint_as_float(u);
}

// sum over each aligned group of G lanes (G a power of two <= 64), the same
// bits in every lane of the group (each step adds two equal partial sums in
// either order); DPP inside a row, ds_bpermute across rows
template <int G>
__device__ __forceinline__ float group_sum(float v) {
  if (G >= 2) v += __uint_as_float(dpp_u32<0xB1>(__float_as_uint(v)));    // lane ^ 1
  if (G >= 4) v += __uint_as_float(dpp_u32<0x4E>(__float_as_uint(v)));    // lane ^ 2
  if (G >= 8) v += __uint_as_float(dpp_u32<0x141>(__float_as_uint(v)));   // row_half_mirror
  if (G >= 16) v += __uint_as_float(dpp_u32<0x140>(__float_as_uint(v)));  // row_mirror
  if (G >= 32) v += __shfl_xor(v, 16, kWave);
  if (G >= 64) v += __shfl_xor(v, 32, kWave);
  return v;
}

// wave-wide sum (all 64 lanes participate)
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
  return v;
}

// Add two per-lane counters to the sharded statistics buffer (kvecc.h): the
// workgroup reduces through LDS and its first lane issues one atomic per
// statistic into slot (blockIdx % KVECC_STATS_SLOTS).  Blocks b and b+8 share
// an XCD under round-robin dispatch, so each slot's adds come from one XCD.
// Must be reached by every thread of the block (it contains a barrier);
// BS = the kernel's block size.
template <int BS = kBlock>
__device__ __forceinline__ void flush_stats2(uint64_t *stats, uint32_t a, uint32_t b) {
  __shared__ uint32_t red[2][BS / kWave];
  a = wave_sum(a);
  b = wave_sum(b);
  const int wave = threadIdx.x / kWave;
  if ((threadIdx.x & (kWave - 1)) == 0) {
    red[0][wave] = a;
    red[1][wave] = b;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long sa = 0, sb = 0;
    for (int w = 0; w < BS / kWave; ++w) {
      sa += red[0][w];
      sb += red[1][w];
    }
    uint64_t *slot = stats + (size_t)(blockIdx.x % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (sa) atomicAdd(reinterpret_cast<unsigned long long *>(slot), sa);
    if (sb) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), sb);
  }
}

// N per-lane counters into words 0..N-1 of the sharded statistics buffer (as
// flush_stats2; one atomic per non-zero statistic per workgroup)
template <int N, int BS = kBlock>
__device__ __forceinline__ void flush_stats_n(uint64_t *stats, const uint32_t (&v)[N]) {
  __shared__ uint32_t red[N][BS / kWave];
  const int wave = threadIdx.x / kWave;
#pragma unroll
  for (int k = 0; k < N; ++k) {
    const uint32_t s = wave_sum(v[k]);
    if ((threadIdx.x & (kWave - 1)) == 0) red[k][wave] = s;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    unsigned long long sum = 0;
    for (int w = 0; w < BS / kWave; ++w) sum += red[threadIdx.x][w];
    uint64_t *slot = stats + (size_t)(blockIdx.x % KVECC_STATS_SLOTS) * KVECC_STATS_STRIDE;
    if (sum) atomicAdd(reinterpret_cast<unsigned long long *>(slot + threadIdx.x), sum);
  }
}

// The dynamic tile schedule of one wave (the fused reads in shim.hip, the
// per-head rows in golay.hip, the packed Golay decode): its first tile is gw,
// next() gives the following ones (>= units: none left).  A wave takes the first
// `pct` % of its even share statically (gw, gw + nwaves, ...), then tiles
// from the launch's work counters: counter c serves the W_c waves gw = c (mod
// kDynCounters) with its K_c tiles (base + k kDynCounters + c); every such wave
// stops after its first failed grab, so the failed grabs return K_c .. K_c +
// W_c - 1, and the wave that draws the last of them is the last to touch the
// counter: it resets it to 0 for the next launch on this counter slot (a "done"
// counter shared by all waves instead serialised their exits: ~40 us).
constexpr uint32_t kTileStaticPct = 75;  // the rows and packed kernels' static share
struct TileSchedule {
  uint32_t gw, nwaves, units, cidx, sidx, gk, last_k, nstatic;
  uint32_t *ctr;
  __device__ __forceinline__ uint32_t grab(uint32_t lane) {
    // the offset is an opaque (per-lane) zero: with a provably uniform address
    // the atomic optimizer rewrites the add into a broadcast of its result
    // right after it, i.e. a vmcnt(0) wait for the round trip on every tile;
    // here the wait comes only where next() reads the value, a tile later
    uint32_t z;
    asm("v_mov_b32 %0, 0" : "=v"(z));
    uint32_t k = 0;
    if (lane == 0) k = __hip_atomic_fetch_add(ctr + z, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return k;  // lane 0's; next() broadcasts it when the tile is needed
  }
  __device__ __forceinline__ void init(uint32_t units_, uint32_t *dyn, uint32_t gw_, uint32_t nwaves_,
                                       uint32_t lane, uint32_t pct = kTileStaticPct) {
    gw = gw_;
    nwaves = nwaves_;
    units = units_;
    sidx = 1;
    // static tiles per wave: pct % of the even share, at least 1
    nstatic = max(1u, (uint32_t)(pct * ((units + nwaves - 1) / nwaves) / 100));
    cidx = gw % kDynCounters;
    ctr = dyn + kDynStride * cidx;
    const uint32_t base = nstatic * nwaves;
    const uint32_t kc = units > base + cidx ? (units - base - cidx + kDynCounters - 1) / kDynCounters : 0u;
    const uint32_t active = min(nwaves, units);  // waves with a first tile (gw < active)
    const uint32_t wc = (active - cidx + kDynCounters - 1) / kDynCounters;  // >= 1: this wave
    last_k = kc + wc - 1;
    gk = grab(lane);
  }
  __device__ __forceinline__ uint32_t next(uint32_t cur, uint32_t lane) {
    (void)cur;
    const uint32_t S = nstatic;
    if (sidx < S) {
      const uint32_t t = gw + sidx * nwaves;
      ++sidx;
      if (t < units) return t;
      sidx = S;
    }
    const uint32_t k = __builtin_amdgcn_readfirstlane(gk);
    const uint32_t t = S * nwaves + k * kDynCounters + cidx;
    if (t < units)
      gk = grab(lane);
    else if (k == last_k && lane == 0)  // the counter's last user
      __hip_atomic_exchange(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return t;
  }
};

// nontemporal streaming load/store helpers (data touched exactly once)
template <typename T>
__device__ __forceinline__ T ld_stream(const T *p) {
  return __builtin_nontemporal_load(p);
}
template <typename T>
__device__ __forceinline__ void st_stream(T *p, T v) {
  __builtin_nontemporal_store(v, p);
}

}  // namespace kvecc
