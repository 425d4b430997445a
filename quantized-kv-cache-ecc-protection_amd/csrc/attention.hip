// attention.hip -- single-token (decode) paged attention over an ECC-protected
// INT4 KV cache, decoding the codewords inline.
//
// Reference: kv_cache/attention_ecc.py:265-427 (paged_attention_ecc_kernel,
// Hamming(8,4) with decode_hamming84_inline :56-149 -- double errors keep their
// uncorrected data -- and dequantize_int4 :152-169) and the wrapper
// paged_attention_ecc :620-780, which the shim calls for seq_len == 1
// (ecc_shim.py:791-800,1091-1136).  Golay(24,12) goes through the Python
// reference_attention_ecc there (:783-909); here it is a native kernel too.
//
// The reference runs one program per (batch, head) walking every context token
// with an online softmax -- B*H programs, a few dozen on a 256-CU part.  This
// is split-context ("flash-decoding"): workgroup (split, b*H + h) owns up to
// 256 tokens (fewer when batch*heads is small, so the grid still fills the
// chip), with the split's slice of the block table staged in LDS.  Lanes are
// grouped W per token row (a lane owns 16 H(8,4) codewords via one 16-byte
// load, or 3 Golay codewords); each group streams its rows in ONE pass --
// kUnroll K and V rows loaded before any is used, the group's partial dot
// products reduced with __shfl_xor, an online softmax per group -- and the
// groups merge through LDS.  The split's (max, sum, acc[D]) go to a workspace
// that a second small launch combines.  Query head h reads cache head
// h / (H / Hkv) (the reference indexes cache head h, which only agrees without
// GQA).  Numerics: fp32 throughout, softmax as exp2 of log2(e)-scaled scores
// (one v_exp_f32 per exponential).  The result differs from the
// reference's sequential online softmax by fp32 summation order and, for Golay,
// by the -8 fold: the kernel sums q*n and p*s*n over the raw nibbles and
// subtracts 8*sum(q) / 8*sum(p*s) once per split (acc - 8*psum), which loses a
// few bits when the values are small against 8*scale (bounded by the
// long-context test in tests/test_attention.py).  A context with no valid
// token (context_len <= 0, or only -1 blocks) gives the reference's values:
// Hamming(8,4) -8.0 in every lane (its kernel scores invalid tokens -1e20, the
// same as its initial max, so each accumulates weight 1 on the masked row
// decode(0) - 8 = -8, attention_ecc.py:342,391-423), Golay 0
// (reference_attention_ecc's torch.zeros, :806-807,885-886).
#include <type_traits>

#include "kvecc_internal.h"

namespace kvecc {

constexpr int kMaxSplit = 1024;   // context tokens per workgroup (upper bound)
constexpr int kMaxSplits = 1024;  // splits per (batch, head)
constexpr int kAttnMaxD = 256;
// Tuned constants (A/B history: DESIGN.md §3 "Paged decode attention";
// tools/exp/run_attn.py and the experiment forks under tools/exp).
// token rows in flight per lane group: packed Golay 4; int32 Golay 2 (72.8 vs
// 80.0 us at 4); Hamming(8,4) 2 (56.9 / 57.1 us vs 60.3 / 60.0 at 4, random /
// encoded caches); every codec loses with 8
constexpr int kUnroll = 4, kGolayUnroll = 2, kH84Unroll = 2;
constexpr int kMaxUnroll = 4;
// codeword words per lane of a token row: H(8,4) 4 (16 codewords, one 16-byte
// load; 8 and 32 per lane measured 57.6 and 65.0 us vs 56.9); Golay 3
// codewords (43 -> 15 of 16 lanes busy; 6 per lane 114.0 vs 104.3 us)
constexpr int kH84Vec = 4, kGolayVec = 3;
// Cache rows go through raw buffer loads with 32-bit offsets when the caches
// and scales are < 4 GiB (the BUF kernels): no 64-bit address arithmetic per
// load, and reads past the row's last codeword need no clamp (inside the
// buffer they read a neighbour row's words, which contribute nothing; past it
// the hardware returns 0).  Golay 105.7 -> 82.1 us at [8,4096,32,128], H84
// unchanged (tools/exp/run_attn.py).  Larger caches take 64-bit addressing.
constexpr uint32_t kRsrcWord3 = 0x00020000u;  // gfx9 raw buffer: 32-bit data format
// Packed Golay caches (KVECC_CODEC_GOLAY_PACKED, 3-byte codewords): a lane owns
// 3 codewords = 9 bytes of its token row, loaded as the 3 aligned dwords that
// hold them and realigned (v_alignbyte): 43 codewords -> 15 of 16 lanes busy.
// 4 codewords per lane (12 bytes, 3 aligned dwords, no realignment) left 5 of
// 16 lanes idle: 68.0 vs 62.8 us per MHA call (profiles/r04/attn/packed_vec_ab.log)
constexpr int kGolayPackedVec = 3;
// Golay decodes through the spread tables (golay_attn_x_table_dev: 32-bit
// entries, nibbles one per byte, parity at the codeword's parity bits): per
// codeword 2 LDS reads + 7 VALU ops (the first table's address, one masked xor
// and a shift for the second's, one masked xor, three v_cvt_f32_ubyteN)
// instead of ~13 through the 16-bit tables.  With the parity at bits 20-31
// (golay_attn_table_dev, the shim's layout) the second address took 3 ops:
// packed MHA main loop 393 -> 357 VALU per 4-row iteration.  Hamming(8,4) decodes through a 256-entry LDS table of data(b) - 8
// as int8 (ds_read_i8 + v_cvt_f32_i32; the 256 bytes are 64 dwords over 32
// banks, so random lookups conflict at most 2-way, where an fp32 table's 256
// dwords conflict ~3.5-way: 60.6 vs 63.5 us per call on random caches).
typedef int8_t h84_lut_t;
// Softmax in base 2: the query is pre-scaled by sm_scale * log2(e), so every
// exponential is one v_exp_f32 (exp2) instead of expf's ~10-instruction range
// reduction (Golay 76.0 -> 72.4 us); the split maxima in the workspace are in
// the same log2 units
__device__ __forceinline__ float attn_exp(float x) { return __builtin_amdgcn_exp2f(x); }  // exp2(-inf) = 0
constexpr float kAttnLogScale = 1.4426950408889634f;  // log2(e)
constexpr bool is_golay(int codec) { return codec == KVECC_CODEC_GOLAY || codec == KVECC_CODEC_GOLAY_PACKED; }

struct AttnArgs {
  const void *q;  // [B, H, D]
  const void *k_cache, *v_cache;
  const int32_t *table;     // [B, max_blocks]
  const int32_t *ctx_lens;  // [B]
  const float *k_scales, *v_scales;
  float *ws;  // [B*H, nsplit, D + 2]: m, l, acc[D]
  void *out;  // [B, H, D]
  int64_t heads, kv_heads, d, g;  // g = codewords per token row
  uint32_t rowb;                  // packed Golay: bytes per token row (KVECC_GOLAY_PACKED_ROW(g))
  int64_t layers, layer, bs, max_blocks, nsplit, split;
  uint32_t cache_bytes, scale_bytes;  // buffer-load bounds (BUF kernels)
  float sm_scale;
  float empty_value;          // output when a (b, h) has no valid token
  const uint16_t *par, *cor;  // Golay tables
  const uint32_t *atab;       // Golay spread tables (golay_attn_table_dev): MFMA kernels
  const uint32_t *atab_x;     // the split kernels' layout (golay_attn_x_table_dev)
  uint32_t *ctr;              // per-(batch, head group) split counters (attn_counter_slot), or
                              // null: a separate combine launch
};

// Lane chunk c of a token row: VEC 32-bit words = 4*VEC H(8,4) codewords, or
// VEC Golay codewords (3*VEC values; codewords past the row's last are read
// clamped and contribute nothing, their values fall outside [0, d)); E values.
template <int CODEC, int VEC>
struct Chunk {
  static constexpr int E = CODEC == KVECC_CODEC_H84 ? 4 * VEC : 3 * VEC;
  // decode() returns (n - 8) + kOffset: the Golay path skips the subtraction
  // per element and the kernel folds -8 * kOffset into the sums instead
  static constexpr float kOffset = is_golay(CODEC) ? 8.0f : 0.0f;
  // Golay: decode() returns value 3k + 2 of each codeword times 16
  static constexpr bool kThird16 = is_golay(CODEC);
  uint32_t w[VEC];
  __device__ __forceinline__ void load_buf(const AttnArgs &a, __amdgpu_buffer_rsrc_t rs, int32_t row,
                                           int c) {
    if constexpr (CODEC == KVECC_CODEC_H84) {
      const uint32_t off = (uint32_t)row * (uint32_t)a.d + 4u * VEC * c;
      if constexpr (VEC % 4 == 0) {
#pragma unroll
        for (int k = 0; k < VEC; k += 4) {
          const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 4 * k, 0, 0));
          w[k] = v.x;
          w[k + 1] = v.y;
          w[k + 2] = v.z;
          w[k + 3] = v.w;
        }
      } else {  // head_dim % 16 != 0: one dword per word (VEC 1 or 2)
#pragma unroll
        for (int k = 0; k < VEC; ++k) w[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4 * k, 0, 0);
      }
    } else if constexpr (CODEC == KVECC_CODEC_GOLAY_PACKED) {
      static_assert(CODEC != KVECC_CODEC_GOLAY_PACKED || VEC == 4 || VEC == 3, "packed lanes own 3 or 4 codewords");
      // past the row's end: a neighbour row's bytes (masked by q = 0) or 0
      if constexpr (VEC == 4) {
        const uint32_t off = (uint32_t)row * a.rowb + 12u * c;
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
        unpack3(v[0], v[1], v[2]);
      } else {  // 9 bytes at 9c: the 3 dwords holding them, realigned.  Rows
                // are whole dwords (KVECC_GOLAY_PACKED_ROW), so the alignment
                // is the lane's own constant, not recomputed per row
        const uint32_t off = (uint32_t)row * a.rowb + ((9u * c) & ~3u);
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
        unpack9(v[0], v[1], v[2], (9u * c) & 3u);
      }
    } else {
      const uint32_t off = ((uint32_t)row * (uint32_t)a.g + VEC * c) * 4u;
      if constexpr (VEC == 3) {  // one 12-byte load: 71.9 vs 72.6 us per MHA call against
                                 // three dword loads (profiles/r06/attn/golay_no_gather_probe.txt)
        const auto v = __builtin_amdgcn_raw_buffer_load_b96(rs, off, 0, 0);
        w[0] = v[0] << 2;
        w[1] = v[1] << 2;
        w[2] = v[2] << 2;
      } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) w[k] = __builtin_amdgcn_raw_buffer_load_b32(rs, off + 4 * k, 0, 0) << 2;
      }
    }
  }
  __device__ __forceinline__ void load(const AttnArgs &a, const void *cache, int64_t row, int c) {
    if constexpr (CODEC == KVECC_CODEC_H84) {
      const uint8_t *p = reinterpret_cast<const uint8_t *>(cache) + row * a.d + 4 * VEC * c;
      if constexpr (VEC % 4 == 0) {
#pragma unroll
        for (int k = 0; k < VEC; k += 4) {
          const u32x4 v = reinterpret_cast<const u32x4 *>(p)[k / 4];
          w[k] = v.x;
          w[k + 1] = v.y;
          w[k + 2] = v.z;
          w[k + 3] = v.w;
        }
      } else {
#pragma unroll
        for (int k = 0; k < VEC; ++k) w[k] = reinterpret_cast<const uint32_t *>(p)[k];
      }
    } else if constexpr (CODEC == KVECC_CODEC_GOLAY_PACKED) {
      const uint32_t *p = reinterpret_cast<const uint32_t *>(reinterpret_cast<const uint8_t *>(cache) + row * a.rowb);
      const int last = (int)(a.rowb / 4) - 1;  // clamp inside the row
      if constexpr (VEC == 4) {
        unpack3(p[min(3 * c, last)], p[min(3 * c + 1, last)], p[min(3 * c + 2, last)]);
      } else {
        const int w0 = 9 * c / 4;
        unpack9(p[min(w0, last)], p[min(w0 + 1, last)], p[min(w0 + 2, last)], (uint32_t)(9 * c) & 3u);
      }
    } else {
      const int32_t *p = reinterpret_cast<const int32_t *>(cache) + row * a.g;
#pragma unroll
      for (int k = 0; k < VEC; ++k) w[k] = (uint32_t)p[min<int64_t>(VEC * c + k, a.g - 1)] << 2;
    }
  }
  // Golay words hold codeword << 2 (bits 0-1 and 26-31: neighbouring bytes,
  // ignored by decode): the first table's byte offset is then one mask.
  // 4 little-endian 3-byte codewords from 3 dwords
  __device__ __forceinline__ void unpack3(uint32_t d0, uint32_t d1, uint32_t d2) {
    w[0] = d0 << 2;
    w[1 < VEC ? 1 : 0] = __builtin_amdgcn_alignbit(d1, d0, 22);
    w[2 < VEC ? 2 : 0] = __builtin_amdgcn_alignbit(d2, d1, 14);
    w[3 < VEC ? 3 : 0] = d2 >> 6;
  }
  // 3 little-endian 3-byte codewords starting at byte `sh` (0-3) of 3 dwords
  __device__ __forceinline__ void unpack9(uint32_t d0, uint32_t d1, uint32_t d2, uint32_t sh) {
    const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sh), x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);
    const uint32_t x2 = d2 >> (8 * sh);
    w[0] = x0 << 2;
    w[1 < VEC ? 1 : 0] = __builtin_amdgcn_alignbit(x1, x0, 22);
    w[2 < VEC ? 2 : 0] = __builtin_amdgcn_alignbit(x2, x1, 14);
  }
  // values before the row scale, (q - 8): H(8,4) through `lut` (LDS, byte ->
  // data(byte) - 8; double errors keep their data, :144-148), Golay through the
  // correction tables (uncorrectable words keep their data, as golay_decode)
  // SP (Golay; instantiated only by tools/exp/attn_exp.hip): the parity half of
  // the spread table as two 64-entry tables, p(lo) = T0[lo & 63] ^ T1[lo >> 6]
  // (the entries are linear in lo), after the 4096-entry correction half: 16.5
  // KiB of LDS instead of 32, conflict-free parity gathers, 2 more VALU per
  // codeword.  Slower at every split and rows-in-flight count tried (MHA
  // int32 75.0 vs 73.2 us, packed 65.2 vs 59.9; profiles/r06/attn/
  // golay_split_parity_ab.txt): the kernel is bound by its VALU work.
  // DEC bits (0: the product; only tools/exp/attn_exp.hip sets any): 1 split
  // parity (SP above), 2 a probe that keeps the decode's VALU but skips its two
  // LDS gathers and the tables' staging and LDS (WRONG values)
  template <int DEC = 0>
  __device__ __forceinline__ void decode(const h84_lut_t *lut, const uint32_t *gtab, float *v) const {
    constexpr bool SP = (DEC & 1) != 0;
    if constexpr (CODEC == KVECC_CODEC_H84) {
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * k + e] = (float)lut[(w[k] >> (8 * e)) & 0xFFu];
      }
    } else {
#pragma unroll
      for (int k = 0; k < VEC; ++k) {
        // w = codeword << 2.  P = golay_attn_x_table_dev[lo] = nibbles 0, 1
        // in bytes 0, 1, nibble 2 in bits 28-31, parity(lo) << 14 -- where w
        // holds the received parity -- so the syndrome's byte offset into the
        // correction half is ((w ^ P) & 0x3FFC000) >> 12: one v_bitop3
        // (0x28 = (S0 ^ S1) & S2) and a shift
        const char *tb = reinterpret_cast<const char *>(gtab);
        uint32_t p;
        if (DEC & 2)
          p = w[k] & 0x3FFCu;
        else if (SP)
          p = *reinterpret_cast<const uint32_t *>(tb + 16384 + (w[k] & 0xFCu)) ^
              *reinterpret_cast<const uint32_t *>(tb + 16384 + 256 + ((w[k] >> 6) & 0xFCu));
        else
          p = *reinterpret_cast<const uint32_t *>(tb + (w[k] & 0x3FFCu));
        const uint32_t off = __builtin_amdgcn_bitop3_b32(w[k], p, 0x03FFC000u, 0x28) >> 12;
        const uint32_t e = (DEC & 2) ? off : *reinterpret_cast<const uint32_t *>(tb + (SP ? 0 : 16384) + off);
        // corrected nibbles: (p ^ e) & 0xF0000F0F; the conversions are written
        // out because the compiler otherwise re-extracts each nibble with a
        // shift and a mask.  The third value comes out as 16 n (byte 3 = n << 4):
        // the kernel prescales its query slot by 1/16 and rescales its
        // accumulator by 1/16 (kThirdScale; powers of two, so exact)
        const uint32_t sp = __builtin_amdgcn_bitop3_b32(p, e, 0xF0000F0Fu, 0x28);
        asm("v_cvt_f32_ubyte0 %0, %1" : "=v"(v[3 * k]) : "v"(sp));  // n, see kOffset
        asm("v_cvt_f32_ubyte1 %0, %1" : "=v"(v[3 * k + 1]) : "v"(sp));
        asm("v_cvt_f32_ubyte3 %0, %1" : "=v"(v[3 * k + 2]) : "v"(sp));  // 16 n
      }
    }
  }
};

typedef float f32x2 __attribute__((ext_vector_type(2)));

// sum_e q[e] * v[e] as packed FMAs (v_pk_fma_f32) into two independent lanes
template <int E>
__device__ __forceinline__ float dot(const float *q, const float *v) {
  f32x2 s = {0.0f, 0.0f};
#pragma unroll
  for (int e = 0; e + 1 < E; e += 2) s = __builtin_elementwise_fma(f32x2{q[e], q[e + 1]}, f32x2{v[e], v[e + 1]}, s);
  if (E % 2) s.x = fmaf(q[E - 1], v[E - 1], s.x);
  return s.x + s.y;
}

// acc[e] += p * v[e] as packed FMAs
template <int E>
__device__ __forceinline__ void axpy(float *acc, float p, const float *v) {
#pragma unroll
  for (int e = 0; e + 1 < E; e += 2) {
    const f32x2 r = __builtin_elementwise_fma(f32x2{p, p}, f32x2{v[e], v[e + 1]}, f32x2{acc[e], acc[e + 1]});
    acc[e] = r.x;
    acc[e + 1] = r.y;
  }
  if (E % 2) acc[E - 1] = fmaf(p, v[E - 1], acc[E - 1]);
}

// Workspace entries under the fused combine are read by a workgroup that may
// sit on another XCD (another L2): they are written and read as agent-scope
// relaxed atomics (global_store / global_load sc1, coherent at the memory side)
// -- an agent-scope fence would write back and invalidate the whole L2
// (buffer_wbl2 / buffer_inv sc1), which measured 4x the kernel's time.
__device__ __forceinline__ void ws_put(float *p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool COHERENT>
__device__ __forceinline__ float ws_get(const float *p) {
  if (COHERENT) return __hip_atomic_load(const_cast<float *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return *p;
}

// combine the splits of one (b, h): out = sum_s acc_s e^(m_s - M) / sum_s l_s e^(m_s - M)
// (one workgroup; wt holds kMaxSplits floats, bred kBlock / kWave).  Two
// "one memory round trip" forms measured slower per 32q/8kv call: every thread
// folding all splits online, one thread per output value (29.5 vs 22.7 us), and
// one wave per (b, h) with the weights by v_readlane (31.2 vs 22.5 us) -- fewer,
// longer-lived waves each walking the splits serially.
template <typename T, bool COHERENT = false>
__device__ void combine_bh(const AttnArgs &a, int64_t bh, float *wt, float *bred) {
  const int64_t stride = a.d + 2;
  const float *ws = a.ws + bh * a.nsplit * stride;
  if (a.nsplit <= kBlock) {
    // one memory round trip: thread s < nsplit loads its split's (m, l) while
    // thread d < head_dim loads its first kPre accumulators; the two block
    // reductions then run in LDS
    constexpr int kPre = 16;
    const int t = threadIdx.x, ns = (int)a.nsplit;
    float ov[kPre];
#pragma unroll
    for (int s = 0; s < kPre; ++s) ov[s] = t < a.d && s < ns ? ws_get<COHERENT>(ws + s * stride + 2 + t) : 0.0f;
    const float ms = t < ns ? ws_get<COHERENT>(ws + t * stride) : -INFINITY;
    const float ls = t < ns ? ws_get<COHERENT>(ws + t * stride + 1) : 0.0f;
    float mx = ms;
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
    if ((t & (kWave - 1)) == 0) bred[t / kWave] = mx;
    __syncthreads();
    mx = bred[0];
#pragma unroll
    for (int w = 1; w < kBlock / kWave; ++w) mx = fmaxf(mx, bred[w]);
    __syncthreads();
    const float w = ms == -INFINITY ? 0.0f : attn_exp(ms - mx);
    if (t < ns) wt[t] = w;
    float L = w * ls;
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) L += __shfl_xor(L, off, kWave);
    if ((t & (kWave - 1)) == 0) bred[t / kWave] = L;
    __syncthreads();
    L = 0.0f;
#pragma unroll
    for (int v = 0; v < kBlock / kWave; ++v) L += bred[v];
    if (t < a.d) {
      float acc = 0.0f;
#pragma unroll
      for (int s = 0; s < kPre; ++s) acc += ov[s] * (s < ns ? wt[s] : 0.0f);
      for (int s = kPre; s < ns; ++s) acc += ws_get<COHERENT>(ws + s * stride + 2 + t) * wt[s];
      reinterpret_cast<T *>(a.out)[bh * a.d + t] = from_f32<T>(L > 0.0f ? acc / L : a.empty_value);
    }
    return;
  }
  float mx = -INFINITY;
  for (int64_t s = threadIdx.x; s < a.nsplit; s += kBlock) mx = fmaxf(mx, ws_get<COHERENT>(ws + s * stride));
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
  if ((threadIdx.x & (kWave - 1)) == 0) bred[threadIdx.x / kWave] = mx;
  __syncthreads();
  mx = bred[0];
#pragma unroll
  for (int w = 1; w < kBlock / kWave; ++w) mx = fmaxf(mx, bred[w]);
  __syncthreads();
  float L = 0.0f;
  for (int64_t s = threadIdx.x; s < a.nsplit; s += kBlock) {
    const float ms = ws_get<COHERENT>(ws + s * stride);
    const float w = ms == -INFINITY ? 0.0f : attn_exp(ms - mx);
    wt[s] = w;
    L += w * ws_get<COHERENT>(ws + s * stride + 1);
  }
#pragma unroll
  for (int off = kWave / 2; off > 0; off >>= 1) L += __shfl_xor(L, off, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0) bred[threadIdx.x / kWave] = L;
  __syncthreads();
  L = 0.0f;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) L += bred[w];
  T *out = reinterpret_cast<T *>(a.out) + bh * a.d;
  for (int64_t di = threadIdx.x; di < a.d; di += kBlock) {
    float acc = 0.0f;
#pragma unroll 4
    for (int64_t s = 0; s < a.nsplit; ++s) acc += ws_get<COHERENT>(ws + s * stride + 2 + di) * wt[s];
    out[di] = from_f32<T>(L > 0.0f ? acc / L : a.empty_value);  // no valid token: see the header
  }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void paged_attn_combine_kernel(AttnArgs a) {
  __shared__ float wt[kMaxSplits];
  __shared__ float bred[kBlock / kWave];
  combine_bh<T>(a, blockIdx.x, wt, bred);
}

// The combine for <= kCombineWaveSplits splits and head_dim <= 128: one
// workgroup of two waves per (b, h), thread d owns output d.  Every wave folds
// the splits' (m, l) itself -- lane s holds split s, the maximum and the
// weighted sum by cross-lane reductions, the weights broadcast by readlane --
// so the kernel has no LDS and no barrier between its one memory round trip
// and its store.
constexpr int kCombineWaveSplits = 16;
template <typename T>
__global__ __launch_bounds__(2 * kWave) void paged_attn_combine_wave_kernel(AttnArgs a) {
  const int64_t bh = blockIdx.x, stride = a.d + 2;
  const float *ws = a.ws + bh * a.nsplit * stride;
  const int t = threadIdx.x, lane = t % kWave, ns = (int)a.nsplit;
  float ov[kCombineWaveSplits];
#pragma unroll
  for (int s = 0; s < kCombineWaveSplits; ++s) ov[s] = t < a.d && s < ns ? ws[s * stride + 2 + t] : 0.0f;
  const float ms = lane < ns ? ws[lane * stride] : -INFINITY;
  const float ls = lane < ns ? ws[lane * stride + 1] : 0.0f;
  float mx = ms;
#pragma unroll
  for (int off = kCombineWaveSplits / 2; off > 0; off >>= 1) mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
  const float w = ms == -INFINITY ? 0.0f : attn_exp(ms - mx);
  float L = w * ls;
#pragma unroll
  for (int off = kCombineWaveSplits / 2; off > 0; off >>= 1) L += __shfl_xor(L, off, kWave);
  L = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, L)));
  if (t < a.d) {
    float acc = 0.0f;
#pragma unroll
    for (int s = 0; s < kCombineWaveSplits; ++s)
      acc += ov[s] * __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, w), s));
    reinterpret_cast<T *>(a.out)[bh * a.d + t] = from_f32<T>(L > 0.0f ? acc / L : a.empty_value);
  }
}

// Fused combine: the workgroup that finishes the last split of its (batch, head
// group) -- counted on a.ctr[blockIdx.y] -- combines the group's G query heads
// and resets the counter, saving the combine launch (the launcher uses it for
// G = 1 only: with G heads the tail after the last split cost more than the
// combine launch, even with all G heads combined in one round trip: 32q/8kv
// 26.7 vs 22.3 us, profiles/r03/attn/attn_gqa19.log).  The workspace stores are
// sc1 (ws_put) and every thread waits for its own before the count; the last
// workgroup reads the entries with sc1 loads.  wt: kMaxSplits floats of LDS the
// caller no longer needs.
//
// Why no release/acquire: on gfx942/gfx950 an sc1 store (ws_put) is performed
// at the memory side (it bypasses the non-coherent per-XCD L2 state for this
// line) once the issuing wave's vmcnt reaches 0, and an sc1 load misses every
// CU/L2 copy, so "store sc1; s_waitcnt vmcnt(0); barrier; atomic add" on the
// writers and "atomic returns the last count; load sc1" on the reader order the
// workspace without the whole-L2 writeback an agent-scope release costs
// (buffer_wbl2: 4x the kernel).  That is a property of these
// targets' cache hierarchy, not of the HIP memory model: any other target must
// not compile this path (the launcher then uses the separate combine kernel).
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "combine_if_last relies on gfx942/gfx950 sc1 + vmcnt ordering; use launch_combine on other targets"
#endif
template <typename T, int G>
__device__ void combine_if_last(const AttnArgs &a, int64_t bh0, float *wt) {
  __shared__ float bred[kBlock / kWave];
  __shared__ uint32_t last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's sc1 workspace stores performed
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t prev = __hip_atomic_fetch_add(a.ctr + blockIdx.y, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = prev + 1 == gridDim.x;
    if (last) __hip_atomic_store(a.ctr + blockIdx.y, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  for (int j = 0; j < G; ++j) {
    if (j) __syncthreads();
    combine_bh<T, true>(a, bh0 + j, wt, bred);
  }
}


// GQA (G > 1): workgroup (split, y) serves the G query heads hg*G .. hg*G+G-1
// of batch b = y / (H/G), which share one cache head: each K and V row is
// loaded and decoded once and used G times (a dot product, an online softmax
// state and an accumulator per head), where one workgroup per query head read
// and decoded every cache row H/Hkv times.
template <typename T, int CODEC, int VEC, int W, bool BUF, int G = 1, int UR = 0, int DEC = 0>
__global__ __launch_bounds__(kBlock) void paged_attn_split_kernel(AttnArgs a) {
  constexpr bool SP = (DEC & 1) != 0;  // Chunk::decode's DEC bits (experiment forks only)
  using C = Chunk<CODEC, VEC>;
  constexpr int E = C::E;
  constexpr int TP = kBlock / W;  // token rows per pass (one per lane group)
  // cache row of each token of the split (-1 = no block / past the split),
  // padded so the unrolled loop reads it without bounds checks
  // (UR > 0: another count, for the experiment forks)
  constexpr int U = UR > 0                        ? UR
                    : CODEC == KVECC_CODEC_GOLAY ? kGolayUnroll
                    : CODEC == KVECC_CODEC_H84   ? kH84Unroll
                                                 : kUnroll;
  static_assert(U <= kMaxUnroll, "rows in flight");
  __shared__ int32_t rows[kMaxSplit + (kMaxUnroll - 1) * kBlock];
  // Golay tables copied from the device: the 32 KiB spread tables, or
  // parity[4096] then correct[4096] as uint16 (16 KiB).  With the spread
  // tables the block-table slice (before the copy) and the merge buffer (after
  // the loop) live in the same LDS, which keeps 4 workgroups per CU.
  constexpr bool kSpread = is_golay(CODEC);
  // (DEC 2, the no-lookup probe: no tables, only the aliased block-table slice and merge buffer)
  constexpr int kProbeWords = TP * W * E > kMaxSplit + 1 ? TP * W * E : kMaxSplit + 1;
  constexpr int kTabWords = !is_golay(CODEC) ? 4 : (DEC & 2) ? kProbeWords : SP ? 4096 + 128 : kSpread ? 8192 : 4096;
  static_assert(!kSpread || (TP * W * E <= kTabWords && kMaxSplit + 1 <= kTabWords), "LDS aliasing");
  __shared__ __attribute__((aligned(16))) uint32_t gtab[kTabWords];
  __shared__ float red_own[kSpread ? 1 : TP * W * E];  // per-group acc
  float *red = kSpread ? reinterpret_cast<float *>(gtab) : red_own;
  __shared__ float gml[2][TP];             // per-group running max / sum
  __shared__ h84_lut_t lut[CODEC == KVECC_CODEC_H84 ? 256 : 1];  // H(8,4): codeword byte -> data - 8

  const int64_t hgroups = a.heads / G;
  const int64_t b = blockIdx.y / hgroups, h0 = (blockIdx.y % hgroups) * G;  // query heads h0 .. h0+G-1
  const int64_t hk = h0 / (a.heads / a.kv_heads);
  const int grp = threadIdx.x / W, c = threadIdx.x % W;
  const int64_t ctx = min<int64_t>(a.ctx_lens[b], a.max_blocks * a.bs);  // table bound
  const int64_t t0 = (int64_t)blockIdx.x * a.split;
  const int64_t t1 = min<int64_t>(t0 + a.split, ctx);
  const int ntok = t1 > t0 ? (int)(t1 - t0) : 0;
  const bool live = c < (a.g + VEC - 1) / VEC;  // lanes past the row idle
  const int cs = live ? c : 0;
  const int64_t ws_stride = a.nsplit * (a.d + 2);  // per query head
  float *ws0 = a.ws + ((b * a.heads + h0) * a.nsplit + blockIdx.x) * (a.d + 2);
  // this lane's query slice, issued before the block-table round trip (first
  // used by the query sums after it)
  float qv[G][E];
  const float qscale = a.sm_scale * kAttnLogScale;
#pragma unroll
  for (int j = 0; j < G; ++j) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int64_t di = (int64_t)c * E + e;
      qv[j][e] = (live && di < a.d)
                     ? to_f32<T>(reinterpret_cast<const T *>(a.q)[(b * a.heads + h0 + j) * a.d + di]) * qscale
                     : 0.0f;
    }
  }

  {  // block-table slice -> LDS (one load per logical block), then one 32-bit
     // division per token; none in the streaming loop
    __shared__ int32_t blks_own[kSpread ? 1 : kMaxSplit + 1];
    int32_t *blks = kSpread ? reinterpret_cast<int32_t *>(gtab) : blks_own;
    const uint32_t bs = (uint32_t)a.bs;
    const uint32_t lb0 = (uint32_t)(t0 / a.bs);
    // the whole split's slice, bounded by the table rather than the context, so
    // the load does not wait for context_lens (one dependent HBM trip fewer)
    const int64_t tmax = min<int64_t>(t0 + a.split, a.max_blocks * a.bs);
    const int nlb = tmax > t0 ? (int)((uint32_t)(tmax - 1) / bs - lb0 + 1) : 0;
    const int32_t *tab = a.table + b * a.max_blocks + lb0;
    for (int j = threadIdx.x; j < nlb; j += kBlock) blks[j] = tab[j];
    __syncthreads();
    const int32_t head_row0 = (int32_t)((a.layer * a.kv_heads + hk) * a.bs);
    const int32_t blk_rows = (int32_t)(a.layers * a.kv_heads * a.bs);
    const int npad = (int)a.split + (U - 1) * kBlock;
    for (int i = threadIdx.x; i < npad; i += kBlock) {
      int32_t row = -1;
      if (i < ntok) {
        const uint32_t pos = (uint32_t)(t0 + i);
        const uint32_t lb = pos / bs;
        const int32_t blk = blks[lb - lb0];
        if (blk >= 0) row = blk * blk_rows + head_row0 + (int32_t)(pos - lb * bs);
      }
      rows[i] = row;
    }
  }
  if (kSpread && (DEC & 2)) {
    __syncthreads();  // blks (aliased) fully read; the probe stages no tables
  } else if (kSpread && SP) {
    __syncthreads();  // blks (aliased) fully read
    // the correction half, then T0[k] = P(k) and T1[k] = P(k << 6)
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a.atab_x + 4096);
    u32x4 *dst = reinterpret_cast<u32x4 *>(gtab);
#pragma unroll
    for (int i = threadIdx.x; i < 1024; i += kBlock) dst[i] = src[i];
    if (threadIdx.x < 128)
      gtab[4096 + threadIdx.x] = a.atab_x[threadIdx.x < 64 ? threadIdx.x : (threadIdx.x - 64) << 6];
  } else if (kSpread) {
    __syncthreads();  // blks (aliased) fully read
    const u32x4 *src = reinterpret_cast<const u32x4 *>(a.atab_x);
    u32x4 *dst = reinterpret_cast<u32x4 *>(gtab);
#pragma unroll
    for (int i = threadIdx.x; i < 2048; i += kBlock) dst[i] = src[i];
  } else if (is_golay(CODEC)) {
    const u32x4 *src0 = reinterpret_cast<const u32x4 *>(a.par);
    const u32x4 *src1 = reinterpret_cast<const u32x4 *>(a.cor);
    u32x4 *dst = reinterpret_cast<u32x4 *>(gtab);
    for (int i = threadIdx.x; i < 512; i += kBlock) {
      dst[i] = src0[i];
      dst[512 + i] = src1[i];
    }
  }
  if (CODEC == KVECC_CODEC_H84 && threadIdx.x < 256) {
    uint32_t q, t, n1 = 0, n2 = 0;
    h84_decode4(threadIdx.x, q, t, n1, n2);
    lut[threadIdx.x] = (h84_lut_t)((int)(q & 0xFu) - 8);
  }
  float qsum[G];  // sum of this lane's q (folds the decode's kOffset out of the K sums)
#pragma unroll
  for (int j = 0; j < G; ++j) {
    qsum[j] = 0.0f;
#pragma unroll
    for (int e = 0; e < E; ++e) qsum[j] += qv[j][e];
    if (C::kThird16) {  // decode's 16 n in slots 3k + 2 (after the sum: it folds n - 8)
#pragma unroll
      for (int e = 2; e < E; e += 3) qv[j][e] *= 0.0625f;
    }
  }
  __syncthreads();

  // buffer descriptors (BUF kernels; dead code otherwise)
  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.k_cache), 0, (int)a.cache_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t vrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.v_cache), 0, (int)a.cache_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t ksrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.k_scales), 0, (int)a.scale_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t vsrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.v_scales), 0, (int)a.scale_bytes, kRsrcWord3);
  // ---- one pass: U K and V rows in flight per lane, online softmax per group
  // (and per query head j of the workgroup)
  float m[G], l[G], acc[G][E];
  float psum[G];  // sum of p * v_scale, for the kOffset fold of the V sums
#pragma unroll
  for (int j = 0; j < G; ++j) {
    m[j] = -INFINITY;
    l[j] = 0.0f;
    psum[j] = 0.0f;
#pragma unroll
    for (int e = 0; e < E; ++e) acc[j][e] = 0.0f;
  }
  // GQA workgroups (G > 1) do G times the arithmetic per row and have a
  // quarter of MHA's rows: they issue the next iteration's rows before using
  // this one's (MHA measured no gain from that in round 1)
  constexpr bool kPrefetch = G > 1 && CODEC == KVECC_CODEC_H84;
  C pkc[U], pvc[U];
  float pks[U], pvs[U];
  bool pok[U];
  auto load_rows = [&](int i0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {  // branch-free: invalid rows read row 0, masked
      const int32_t r = rows[i0 + u * TP];
      pok[u] = r >= 0;
      const int64_t row = pok[u] ? r : 0;
      if (BUF) {
        pkc[u].load_buf(a, krs, (int32_t)row, cs);
        pvc[u].load_buf(a, vrs, (int32_t)row, cs);
        pks[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ksrs, (uint32_t)row * 4u, 0, 0));
        pvs[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vsrs, (uint32_t)row * 4u, 0, 0));
      } else {
        pkc[u].load(a, a.k_cache, row, cs);
        pvc[u].load(a, a.v_cache, row, cs);
        pks[u] = a.k_scales[row];
        pvs[u] = a.v_scales[row];
      }
    }
  };
  if (kPrefetch && grp < ntok) load_rows(grp);
  for (int i0 = grp; i0 < ntok; i0 += TP * U) {
    if (!kPrefetch) load_rows(i0);
    C kc[U], vc[U];
    float ks[U], vs[U];
    bool ok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      kc[u] = pkc[u];
      vc[u] = pvc[u];
      ks[u] = pks[u];
      vs[u] = pvs[u];
      ok[u] = pok[u];
    }
    if (kPrefetch && i0 + TP * U < ntok) load_rows(i0 + TP * U);
    float sc[G][U];
    float mn[G];
#pragma unroll
    for (int j = 0; j < G; ++j) mn[j] = m[j];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float part[G];
#pragma unroll
      for (int j = 0; j < G; ++j) part[j] = 0.0f;
      if (live) {
        float kv[E];
        kc[u].template decode<DEC>(lut, gtab, kv);
#pragma unroll
        for (int j = 0; j < G; ++j) {
          part[j] = dot<E>(qv[j], kv);
          if (C::kOffset != 0.0f) part[j] -= C::kOffset * qsum[j];
          part[j] *= ks[u];  // sum q (n - 8) s = s * sum q (n - 8)
        }
      }
#pragma unroll
      for (int j = 0; j < G; ++j) {
        part[j] = group_sum<W>(part[j]);
        sc[j][u] = ok[u] ? part[j] : -INFINITY;
        mn[j] = fmaxf(mn[j], sc[j][u]);
      }
    }
    bool any = false;
#pragma unroll
    for (int j = 0; j < G; ++j) any |= mn[j] != -INFINITY;
    if (!any) continue;  // no valid row yet (uniform per group)
    float ps[G][U];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      if (G > 1 && mn[j] == -INFINITY) {  // this head has no finite score yet: no update
#pragma unroll
        for (int u = 0; u < U; ++u) ps[j][u] = 0.0f;
        continue;
      }
      const float alpha = attn_exp(m[j] - mn[j]);  // m = -inf -> 0
      l[j] *= alpha;
      psum[j] *= alpha;
#pragma unroll
      for (int e = 0; e < E; ++e) acc[j][e] *= alpha;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float p = attn_exp(sc[j][u] - mn[j]);  // invalid rows: exp(-inf) = 0
        l[j] += p;
        ps[j][u] = p * vs[u];
        psum[j] += ps[j][u];
      }
      m[j] = mn[j];
    }
    if (live) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float vv[E];
        vc[u].template decode<DEC>(lut, gtab, vv);
#pragma unroll
        for (int j = 0; j < G; ++j) axpy<E>(acc[j], ps[j][u], vv);
      }
    }
  }

  // ---- merge the TP groups (one query head at a time) ------------------------------
  if (kSpread) __syncthreads();  // the tables (aliased by red) fully read
  __shared__ float gw[TP];  // e^(m_g - M) per group
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if (j > 0) __syncthreads();  // the previous head's merge fully read red / gml / gw
    if (live) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float ae = C::kThird16 && e % 3 == 2 ? acc[j][e] * 0.0625f : acc[j][e];  // 16 n slots
        red[(grp * W + c) * E + e] = C::kOffset != 0.0f ? ae - C::kOffset * psum[j] : ae;
      }
    }
    if (c == 0) {
      gml[0][grp] = m[j];
      gml[1][grp] = l[j];
    }
    __syncthreads();
    float M = -INFINITY;
    for (int gi = 0; gi < TP; ++gi) M = fmaxf(M, gml[0][gi]);
    if (threadIdx.x < TP) {
      const float mg = gml[0][threadIdx.x];
      gw[threadIdx.x] = mg == -INFINITY ? 0.0f : attn_exp(mg - M);
    }
    __syncthreads();
    float *ws = ws0 + j * ws_stride;
    for (int64_t di = threadIdx.x; di < a.d; di += kBlock) {
      float sum = 0.0f;
      for (int gi = 0; gi < TP; ++gi) sum += red[gi * W * E + di] * gw[gi];
      ws_put(ws + 2 + di, sum);
    }
    if (threadIdx.x == 0) {
      float L = 0.0f;
      for (int gi = 0; gi < TP; ++gi) L += gml[1][gi] * gw[gi];
      ws_put(ws, M);
      ws_put(ws + 1, L);
    }
  }
  if (a.ctr) combine_if_last<T, G>(a, b * a.heads + h0, reinterpret_cast<float *>(rows));
}

// ---- GQA on the matrix cores (Hamming(8,4), fp16 queries) -----------------------
//
// With G query heads per cache head the VALU kernel above does G dot products
// and G accumulator updates per decoded value, so its time stays near the MHA
// kernel's while the cache bytes fall by G.  Here both products run on
// v_mfma_f32_16x16x32_f16, and the VALU only decodes:
//   S^T[16 tokens x 16 heads] = K[16 tokens x D] . Q^T[D x 16 heads]   (D/32 MFMAs per 16 tokens)
//   O^T[16 d x 16 heads]     += V^T[16 d x 32 tokens] . P[32 tokens x 16 heads]
// Columns are query heads (G <= 16 used, the rest zero).  Decoded values n - 8
// (integers in [-8, 7]) and the fp16 queries are exact in f16, so the scores
// are the fp32 sums of exact products, as in the VALU kernel; P (fp32) goes
// in as two f16 halves, hi + lo, 22 bits.  The operand maps (A[row l&15][k =
// 8(l>>4)+j], B[k][col l&15], C[row 4(l>>4)+r][col l&15]) are bent so that
// every lane's loads stay contiguous and no value moves between lanes:
//   * K: lane (token t = l&15, group g = l>>4) loads D/4 contiguous bytes of its
//     token row, d = (D/4)g .. ; MFMA kk takes bytes 8kk..8kk+7 (the same k -> d
//     map for the Q operand, which is loaded once);
//   * a wave step is 32 tokens, two S^T tiles; lane (head n, g) then holds
//     the scores of tokens 4g + r and 16 + 4g + r (r = 0..3) for head n -- which
//     are exactly the 8 k-slots of the PV B operand when PV's k maps slot
//     8g + j to token 16(j >> 2) + 4g + (j & 3): P needs no shuffle;
//   * V: the same 8 tokens per lane, D/16 contiguous bytes each at d = (D/16) m
//     (m = l&15); M-tile mt takes byte mt of each, so output row m of tile mt
//     is d = (D/16)(4g + r) + mt.
// Decode: LDS table byte -> data nibble (single errors corrected, doubles keep
// their data, attention_ecc.py:56-149), pairs packed as f16 1024 + n by an OR
// of 0x6400 and shifted by one v_pk_add_f16 of -1032.  The online softmax runs
// per lane on its 8 scores (head maxima across the 4 lanes of a head with two
// xor-shuffles), the workgroup's 4 waves merge through LDS, and the split goes
// to the workspace of the combine kernel above.
// Fused combine: the last split of each (batch, head group) combines it
// (combine_if_last) -- for one query head per workgroup only (see
// kvecc_paged_attention).  Issuing the next step's loads before this step's
// math took the kernel to 191 VGPRs (2 waves per SIMD): 32q/8kv 29.8 us
// against 22.9 without.  4 workgroups per CU for the H(8,4) kernel.
constexpr int kMfmaWgPerCu = 4;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int kMfmaStep = 32;  // tokens per wave step

// Decoded values as MFMA operands: the table's nibble n (0..15) goes into an
// f16 half as is -- the subnormal n * 2^-24, exact -- so a pair costs one
// v_perm; the kernel scales the products by 2^24 and folds the -8 out as
// -8 * sum(q) (scores) and -8 * sum(p) (outputs).  (f16 1024 + n by an OR of
// 0x6400 and one v_pk_add_f16 of -1032 per pair measured within noise.)
constexpr float kMfmaValScale = 16777216.0f;  // 2^24
constexpr float kMfmaValOffset = 8.0f;
// two table values (data nibbles 0..15) -> f16 operand pair, lo in bits 0..15
__device__ __forceinline__ uint32_t nib_pair_f16(uint32_t lo, uint32_t hi) {
  return __builtin_amdgcn_perm(hi, lo, 0x0c040c00u);  // [0, hi, 0, lo]
}

// NB contiguous bytes (2, 4, 8, 16 or 32) at byte offset off -> dwords w
template <int NB>
__device__ __forceinline__ void load_chunk(__amdgpu_buffer_rsrc_t rs, uint32_t off, uint32_t *w) {
  if constexpr (NB == 2) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0);
  } else if constexpr (NB == 4) {
    w[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0);
  } else if constexpr (NB == 8) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0);
    w[0] = v[0];
    w[1] = v[1];
  } else {
#pragma unroll
    for (int k = 0; k < NB / 16; ++k) {
      const u32x4 v = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16 * k, 0, 0));
      w[4 * k] = v.x;
      w[4 * k + 1] = v.y;
      w[4 * k + 2] = v.z;
      w[4 * k + 3] = v.w;
    }
  }
}

template <int D, int G>
__global__ __launch_bounds__(kBlock, 2) void paged_attn_h84_mfma_kernel(AttnArgs a) {
  constexpr int KK = D / 32;  // QK MFMAs per 16-token tile
  constexpr int MT = D / 16;  // PV M-tiles; V bytes per lane per token
  constexpr int KB = D / 4;   // K bytes per lane per token
  constexpr int VW = MT >= 4 ? MT / 4 : 1;  // V dwords per token
  constexpr int kWaves = kBlock / kWave;
  __shared__ __attribute__((aligned(16))) int32_t rows[kMaxSplit + kMfmaStep];
  __shared__ int32_t blks[kMaxSplit + 1];
  __shared__ uint8_t lut[256];
  __shared__ float red[kWaves][G][D];
  __shared__ float gml[2][kWaves][G];

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int n = lane & 15, g = lane >> 4;
  const int64_t hgroups = a.heads / G;
  const int64_t b = blockIdx.y / hgroups, h0 = (blockIdx.y % hgroups) * G;
  const int64_t hk = h0 / (a.heads / a.kv_heads);
  const int64_t ctx = min<int64_t>(a.ctx_lens[b], a.max_blocks * a.bs);
  const int64_t t0 = (int64_t)blockIdx.x * a.split;
  const int64_t t1 = min<int64_t>(t0 + a.split, ctx);
  const int ntok = t1 > t0 ? (int)(t1 - t0) : 0;
  // Q^T operand (B): column n = head h0 + n, k-slot 8g + j of MFMA kk = d (D/4)g + 8kk + j.
  // Issued first: it lands during the block-table round trip instead of
  // after it (its first use, the query sum, precedes the first K/V loads)
  f16x8 qop[KK];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    u32x4 v = {0u, 0u, 0u, 0u};
    if (n < G)
      v = *reinterpret_cast<const u32x4 *>(reinterpret_cast<const __half *>(a.q) +
                                           (b * a.heads + h0 + n) * D + KB * g + 8 * kk);
    qop[kk] = __builtin_bit_cast(f16x8, v);
  }
  {  // block-table slice -> cache rows (-1: no block / past the split)
    const uint32_t bs = (uint32_t)a.bs;
    const uint32_t lb0 = (uint32_t)(t0 / a.bs);
    // the whole split's slice, bounded by the table rather than the context, so
    // the load does not wait for context_lens (one dependent HBM trip fewer)
    const int64_t tmax = min<int64_t>(t0 + a.split, a.max_blocks * a.bs);
    const int nlb = tmax > t0 ? (int)((uint32_t)(tmax - 1) / bs - lb0 + 1) : 0;
    const int32_t *tab = a.table + b * a.max_blocks + lb0;
    for (int j = threadIdx.x; j < nlb; j += kBlock) blks[j] = tab[j];
    __syncthreads();
    const int32_t head_row0 = (int32_t)((a.layer * a.kv_heads + hk) * a.bs);
    const int32_t blk_rows = (int32_t)(a.layers * a.kv_heads * a.bs);
    const int npad = (ntok + kMfmaStep - 1) / kMfmaStep * kMfmaStep;
    for (int i = threadIdx.x; i < npad; i += kBlock) {
      int32_t row = -1;
      if (i < ntok) {
        const uint32_t pos = (uint32_t)(t0 + i);
        const uint32_t lb = pos / bs;
        const int32_t blk = blks[lb - lb0];
        if (blk >= 0) row = blk * blk_rows + head_row0 + (int32_t)(pos - lb * bs);
      }
      rows[i] = row;
    }
  }
  {
    uint32_t dq, dt, n1 = 0, n2 = 0;
    h84_decode4(threadIdx.x, dq, dt, n1, n2);  // kBlock == 256: one table entry per thread
    lut[threadIdx.x] = (uint8_t)(dq & 0xFu);
  }
  float qsum = 0.0f;  // sum of head n's query over all d (the offset fold)
#pragma unroll
  for (int kk = 0; kk < KK; ++kk)
#pragma unroll
    for (int e = 0; e < 8; ++e) qsum += (float)qop[kk][e];
  qsum += __shfl_xor(qsum, 16, kWave);
  qsum += __shfl_xor(qsum, 32, kWave);
  __syncthreads();

  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.k_cache), 0, (int)a.cache_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t vrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.v_cache), 0, (int)a.cache_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t ksrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.k_scales), 0, (int)a.scale_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t vsrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.v_scales), 0, (int)a.scale_bytes, kRsrcWord3);
  const float qscale = a.sm_scale * kAttnLogScale;
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float m = -INFINITY, l = 0.0f;
  float psum = 0.0f;  // sum of p * v_scale over this lane's tokens (the offset fold)
  const float qoff = kMfmaValOffset * qsum;

  // one step's operands in registers: 2 K rows (tokens i0 + n, i0 + 16 + n),
  // 8 V rows and scales (tokens i0 + 16(j >> 2) + 4g + (j & 3)); invalid rows
  // read row 0 and are masked
  struct Step {
    int32_t rv[8];
    uint32_t kw[2][KB / 4 > 0 ? KB / 4 : 1];
    uint32_t vw[8][VW];
    float ks[8], vs[8];
  };
  auto load_step = [&](int i0, Step &st) {
    const int4 r0 = *reinterpret_cast<const int4 *>(&rows[i0 + 4 * g]);
    const int4 r1 = *reinterpret_cast<const int4 *>(&rows[i0 + 16 + 4 * g]);
    st.rv[0] = r0.x; st.rv[1] = r0.y; st.rv[2] = r0.z; st.rv[3] = r0.w;
    st.rv[4] = r1.x; st.rv[5] = r1.y; st.rv[6] = r1.z; st.rv[7] = r1.w;
#pragma unroll
    for (int tau = 0; tau < 2; ++tau) {
      const int32_t r = rows[i0 + 16 * tau + n];
      load_chunk<KB>(krs, (uint32_t)max(r, 0) * (uint32_t)D + (uint32_t)(KB * g), st.kw[tau]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t r = (uint32_t)max(st.rv[j], 0);
      load_chunk<MT>(vrs, r * (uint32_t)D + (uint32_t)(MT * n), st.vw[j]);
      st.ks[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ksrs, r * 4u, 0, 0));
      st.vs[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vsrs, r * 4u, 0, 0));
    }
  };
  constexpr int kStride = kWaves * kMfmaStep;
  for (int i0 = wave * kMfmaStep; i0 < ntok; i0 += kStride) {
    Step cur;
    load_step(i0, cur);
    const int32_t *rv = cur.rv;
    const float *ks = cur.ks, *vs = cur.vs;
    auto &kw = cur.kw;
    auto &vw = cur.vw;
    // ---- S^T = K . Q^T, two 16-token tiles
    f32x4 S[2];
#pragma unroll
    for (int tau = 0; tau < 2; ++tau) {
      S[tau] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        uint32_t p[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {  // bytes 8kk + 2h, 8kk + 2h + 1
          const uint32_t w = kw[tau][2 * kk + h / 2];
          const int sh = 16 * (h & 1);
          p[h] = nib_pair_f16(lut[(w >> sh) & 0xFFu], lut[(w >> (sh + 8)) & 0xFFu]);
        }
        S[tau] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, u32x4{p[0], p[1], p[2], p[3]}),
                                                        qop[kk], S[tau], 0, 0, 0);
      }
    }
    // ---- online softmax over this lane's 8 tokens of head n
    float s[8];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] = rv[j] >= 0 ? (S[j >> 2][j & 3] * kMfmaValScale - qoff) * (qscale * ks[j]) : -INFINITY;
      mx = fmaxf(mx, s[j]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
    mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
    const float mn = fmaxf(m, mx);
    const float mu = mn == -INFINITY ? 0.0f : mn;  // no valid token yet: nothing to scale
    const float alpha = attn_exp(m - mu);
    m = mn;
    l *= alpha;
    psum *= alpha;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] *= alpha;
    uint32_t phi[4], plo[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const float p0 = attn_exp(s[2 * h] - mu), p1 = attn_exp(s[2 * h + 1] - mu);
      l += p0 + p1;
      const float w0 = p0 * vs[2 * h], w1 = p1 * vs[2 * h + 1];
      psum += w0 + w1;
      const auto hi = __builtin_amdgcn_cvt_pkrtz(w0, w1);
      const auto lo = __builtin_amdgcn_cvt_pkrtz(w0 - (float)hi[0], w1 - (float)hi[1]);
      phi[h] = __builtin_bit_cast(uint32_t, hi);
      plo[h] = __builtin_bit_cast(uint32_t, lo);
    }
    const f16x8 pb_hi = __builtin_bit_cast(f16x8, u32x4{phi[0], phi[1], phi[2], phi[3]});
    const f16x8 pb_lo = __builtin_bit_cast(f16x8, u32x4{plo[0], plo[1], plo[2], plo[3]});
    // ---- O^T += V^T . P: M-tile mt takes byte mt of each token's chunk
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      uint32_t p[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) {  // tokens j = 2h, 2h + 1
        const int sh = 8 * (mt & 3);
        p[h] = nib_pair_f16(lut[(vw[2 * h][mt / 4] >> sh) & 0xFFu], lut[(vw[2 * h + 1][mt / 4] >> sh) & 0xFFu]);
      }
      const f16x8 va = __builtin_bit_cast(f16x8, u32x4{p[0], p[1], p[2], p[3]});
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb_hi, acc[mt], 0, 0, 0);
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb_lo, acc[mt], 0, 0, 0);
    }
  }

  // ---- merge: the 4 lanes of a head, then the workgroup's waves
  l += __shfl_xor(l, 16, kWave);
  l += __shfl_xor(l, 32, kWave);
  psum += __shfl_xor(psum, 16, kWave);
  psum += __shfl_xor(psum, 32, kWave);
  const float poff = kMfmaValOffset * psum;
  if (n < G) {
    if (g == 0) {
      gml[0][wave][n] = m;
      gml[1][wave][n] = l;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wave][n][MT * (4 * g + r) + mt] = acc[mt][r] * kMfmaValScale - poff;
  }
  __syncthreads();
  const int64_t ws_stride = a.nsplit * (a.d + 2);
  float *ws0 = a.ws + ((b * a.heads + h0) * a.nsplit + blockIdx.x) * (a.d + 2);
  for (int idx = threadIdx.x; idx < G * D; idx += kBlock) {
    const int h = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) M = fmaxf(M, gml[0][w][h]);
    float o = 0.0f, L = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const float mw = gml[0][w][h];
      const float wt = mw == -INFINITY ? 0.0f : attn_exp(mw - M);
      o += red[w][h][d] * wt;
      L += gml[1][w][h] * wt;
    }
    float *ws = ws0 + h * ws_stride;
    ws_put(ws + 2 + d, o);
    if (d == 0) {
      ws_put(ws, M);
      ws_put(ws + 1, L);
    }
  }
  if (a.ctr) combine_if_last<__half, G>(a, b * a.heads + h0, reinterpret_cast<float *>(rows));
}

// ---- GQA on the matrix cores, Golay(24,12) int32 caches, head_dim 128 ---------
//
// The H(8,4) kernel's scheme with codeword-aligned operand maps (a row is 43
// codewords = 129 nibbles, d = 3c + e):
//   * QK: lane group g owns codewords 11g .. 11g+10 of its token's K row (44
//     bytes: two 16-byte loads and a 12-byte one), i.e. d = 33g .. 33g+32, as
//     k-slots 0..32 of 40 (5 MFMAs per 16 tokens; slots past 32, and d >= 128,
//     carry q = 0);
//   * PV: lane m owns codewords 3m .. 3m+2 (a 12-byte load per token), 9
//     M-tiles, output row m of tile mt is d = 9m + mt (d >= 128 discarded).
// Codewords decode through the spread tables (two LDS reads, one v_bitop3) to
// nibbles one per byte; an operand pair is one v_perm of two decoded words
// into f16 subnormals (n * 2^-24), with the 2^24 scale and the -8 folds of the
// H(8,4) kernel.  Tokens, scales, the softmax and the merge are that kernel's.
//
// Packed caches (3-byte codewords, 132-byte rows) keep the maps where the loads
// stay dword-aligned: K lane groups own 12 codewords (36 bytes at 36g, d = 36g
// .. 36g+35, still 5 MFMAs), V lanes own codewords 3m .. 3m+2 (9 bytes at 9m:
// one 12-byte load from the dword below, then v_alignbyte by m & 3).  Bytes past
// the row's 129 belong to d >= 128 (q = 0, outputs discarded).
template <int G, bool PACKED>
__global__ __launch_bounds__(kBlock, 2) void paged_attn_golay_mfma_kernel(AttnArgs a) {
  constexpr int D = 128, GC = 43;          // head_dim, codewords per row
  constexpr int KC = PACKED ? 12 : 11;     // K codewords per lane group
  constexpr int KD = 3 * KC, KK = 5;       // its values; QK MFMAs per 16 tokens
  constexpr int VC = 3, MT = 9;            // V codewords per lane; PV M-tiles
  constexpr int KW = PACKED ? 9 : KC;      // K dwords per lane group
  constexpr uint32_t kRowBytes = PACKED ? KVECC_GOLAY_PACKED_ROW(GC) : GC * 4;
  constexpr int kWaves = kBlock / kWave;
  __shared__ __attribute__((aligned(16))) uint32_t gt[8192];  // spread tables (golay_attn_table_dev)
  __shared__ __attribute__((aligned(16))) int32_t rows[kMaxSplit + kMfmaStep];
  __shared__ int32_t blks[kMaxSplit + 1];
  __shared__ float red[kWaves][G][D];
  __shared__ float gml[2][kWaves][G];

  const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
  const int n = lane & 15, g = lane >> 4;
  const int64_t hgroups = a.heads / G;
  const int64_t b = blockIdx.y / hgroups, h0 = (blockIdx.y % hgroups) * G;
  const int64_t hk = h0 / (a.heads / a.kv_heads);
  const int64_t ctx = min<int64_t>(a.ctx_lens[b], a.max_blocks * a.bs);
  const int64_t t0 = (int64_t)blockIdx.x * a.split;
  const int64_t t1 = min<int64_t>(t0 + a.split, ctx);
  const int ntok = t1 > t0 ? (int)(t1 - t0) : 0;
  // Q^T operand: k-slot v = 8kk + j of lane group g is d = KD g + v (v < KD, d < 128), else 0;
  // issued before the block-table round trip, as in the H(8,4) kernel
  f16x8 qop[KK];
  {
    const __half *qh = reinterpret_cast<const __half *>(a.q) + (b * a.heads + h0 + n) * D;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int v = 8 * kk + j, d = KD * g + v;
        _Float16 x = 0;
        if (n < G && v < KD && d < D) x = __builtin_bit_cast(_Float16, qh[d]);
        qop[kk][j] = x;
      }
    }
  }
  {  // block-table slice -> cache rows, as in the H(8,4) kernel
    const uint32_t bs = (uint32_t)a.bs;
    const uint32_t lb0 = (uint32_t)(t0 / a.bs);
    const int64_t tmax = min<int64_t>(t0 + a.split, a.max_blocks * a.bs);
    const int nlb = tmax > t0 ? (int)((uint32_t)(tmax - 1) / bs - lb0 + 1) : 0;
    const int32_t *tab = a.table + b * a.max_blocks + lb0;
    for (int j = threadIdx.x; j < nlb; j += kBlock) blks[j] = tab[j];
    {
      const u32x4 *src = reinterpret_cast<const u32x4 *>(a.atab);
      for (int i = threadIdx.x; i < 2048; i += kBlock) reinterpret_cast<u32x4 *>(gt)[i] = src[i];
    }
    __syncthreads();
    const int32_t head_row0 = (int32_t)((a.layer * a.kv_heads + hk) * a.bs);
    const int32_t blk_rows = (int32_t)(a.layers * a.kv_heads * a.bs);
    const int npad = (ntok + kMfmaStep - 1) / kMfmaStep * kMfmaStep;
    for (int i = threadIdx.x; i < npad; i += kBlock) {
      int32_t row = -1;
      if (i < ntok) {
        const uint32_t pos = (uint32_t)(t0 + i);
        const uint32_t lb = pos / bs;
        const int32_t blk = blks[lb - lb0];
        if (blk >= 0) row = blk * blk_rows + head_row0 + (int32_t)(pos - lb * bs);
      }
      rows[i] = row;
    }
  }
  float qsum = 0.0f;
  {
#pragma unroll
    for (int kk = 0; kk < KK; ++kk)
#pragma unroll
      for (int j = 0; j < 8; ++j) qsum += (float)qop[kk][j];
    qsum += __shfl_xor(qsum, 16, kWave);
    qsum += __shfl_xor(qsum, 32, kWave);
  }
  __syncthreads();

  // codeword -> data nibbles one per byte (bytes 0..2), uncorrectable words keep
  // their data.  (The split kernels' table, parity at the codeword's parity
  // bits and the nibbles in bytes 0, 1, 3, measured 1 % slower here:
  // profiles/r04/attn/xtab_ab.log.)
  auto sp_of = [&](uint32_t c) -> uint32_t {
    const uint32_t p = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(gt) + ((c << 2) & 0x3FFCu));
    const uint32_t off = ((c >> 10) ^ (p >> 18)) & 0x3FFCu;
    const uint32_t e = *reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(gt + 4096) + off);
    return __builtin_amdgcn_bitop3_b32(p, e, 0x000F0F0Fu, 0x28);  // (p ^ e) & mask
  };
  // f16 subnormal pair: byte e0 of lo (0x0c: zero), byte e1 of hi, in halves 0 and 1
  auto pair = [](uint32_t hi, uint32_t lo, int e0, int e1) -> uint32_t {
    const uint32_t s0 = e0 < 0 ? 0x0cu : (uint32_t)e0, s1 = e1 < 0 ? 0x0cu : (uint32_t)(4 + e1);
    return __builtin_amdgcn_perm(hi, lo, 0x0c000c00u | s1 << 16 | s0);
  };

  const __amdgpu_buffer_rsrc_t krs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.k_cache), 0, (int)a.cache_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t vrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(a.v_cache), 0, (int)a.cache_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t ksrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.k_scales), 0, (int)a.scale_bytes, kRsrcWord3);
  const __amdgpu_buffer_rsrc_t vsrs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(a.v_scales), 0, (int)a.scale_bytes, kRsrcWord3);
  constexpr float kScale = 16777216.0f, kOff = 8.0f;  // subnormal operands: 2^24, and n - 8
  const float qscale = a.sm_scale * kAttnLogScale;
  const float qoff = kOff * qsum;
  f32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
  float m = -INFINITY, l = 0.0f, psum = 0.0f;

  for (int i0 = wave * kMfmaStep; i0 < ntok; i0 += kWaves * kMfmaStep) {
    int32_t rv[8];
    {
      const int4 r0 = *reinterpret_cast<const int4 *>(&rows[i0 + 4 * g]);
      const int4 r1 = *reinterpret_cast<const int4 *>(&rows[i0 + 16 + 4 * g]);
      rv[0] = r0.x; rv[1] = r0.y; rv[2] = r0.z; rv[3] = r0.w;
      rv[4] = r1.x; rv[5] = r1.y; rv[6] = r1.z; rv[7] = r1.w;
    }
    uint32_t kw[2][KW];
#pragma unroll
    for (int tau = 0; tau < 2; ++tau) {
      const uint32_t off = (uint32_t)max(rows[i0 + 16 * tau + n], 0) * kRowBytes + 4u * KW * g;
      const u32x4 x0 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, off, 0, 0));
      const u32x4 x1 = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(krs, off + 16, 0, 0));
      kw[tau][0] = x0.x; kw[tau][1] = x0.y; kw[tau][2] = x0.z; kw[tau][3] = x0.w;
      kw[tau][4] = x1.x; kw[tau][5] = x1.y; kw[tau][6] = x1.z; kw[tau][7] = x1.w;
      if constexpr (PACKED) {
        kw[tau][8] = __builtin_amdgcn_raw_buffer_load_b32(krs, off + 32, 0, 0);
      } else {
        const auto x2 = __builtin_amdgcn_raw_buffer_load_b96(krs, off + 32, 0, 0);
        kw[tau][8] = x2[0]; kw[tau][9] = x2[1]; kw[tau][10] = x2[2];
      }
    }
    // V: this lane's codewords start 12n bytes (int32) or 9n bytes (packed) into the row
    const uint32_t voff = PACKED ? (9u * n) & ~3u : 12u * n;
    const uint32_t vsh = n & 3;  // packed: byte of the first codeword in the loaded dword
    uint32_t vw[8][VC];
    float ks[8], vs[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t r = (uint32_t)max(rv[j], 0);
      const auto x = __builtin_amdgcn_raw_buffer_load_b96(vrs, r * kRowBytes + voff, 0, 0);
      vw[j][0] = x[0]; vw[j][1] = x[1]; vw[j][2] = x[2];
      ks[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(ksrs, r * 4u, 0, 0));
      vs[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(vsrs, r * 4u, 0, 0));
    }
    // ---- S^T = K . Q^T
    f32x4 S[2];
#pragma unroll
    for (int tau = 0; tau < 2; ++tau) {
      uint32_t cw[KC];
      if constexpr (PACKED) {  // 4 little-endian 3-byte codewords per 3 dwords
#pragma unroll
        for (int t = 0; t < 3; ++t) {
          const uint32_t d0 = kw[tau][3 * t], d1 = kw[tau][3 * t + 1], d2 = kw[tau][3 * t + 2];
          cw[4 * t] = d0;
          cw[4 * t + 1] = __builtin_amdgcn_alignbyte(d1, d0, 3);
          cw[4 * t + 2] = __builtin_amdgcn_alignbyte(d2, d1, 2);
          cw[4 * t + 3] = d2 >> 8;
        }
      } else {
#pragma unroll
        for (int c = 0; c < KC; ++c) cw[c] = kw[tau][c];
      }
      uint32_t sp[KC];
#pragma unroll
      for (int c = 0; c < KC; ++c) sp[c] = sp_of(cw[c]);
      S[tau] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        uint32_t p[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const int v0 = 8 * kk + 2 * h, v1 = v0 + 1;
          const int c0 = v0 < KD ? v0 / 3 : 0, c1 = v1 < KD ? v1 / 3 : 0;
          p[h] = pair(sp[c1], sp[c0], v0 < KD ? v0 % 3 : -1, v1 < KD ? v1 % 3 : -1);
        }
        S[tau] = __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, u32x4{p[0], p[1], p[2], p[3]}),
                                                        qop[kk], S[tau], 0, 0, 0);
      }
    }
    // ---- online softmax over this lane's 8 tokens of head n
    float s[8];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] = rv[j] >= 0 ? (S[j >> 2][j & 3] * kScale - qoff) * (qscale * ks[j]) : -INFINITY;
      mx = fmaxf(mx, s[j]);
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
    mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
    const float mn = fmaxf(m, mx);
    const float mu = mn == -INFINITY ? 0.0f : mn;
    const float alpha = attn_exp(m - mu);
    m = mn;
    l *= alpha;
    psum *= alpha;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] *= alpha;
    uint32_t phi[4], plo[4];
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const float p0 = attn_exp(s[2 * h] - mu), p1 = attn_exp(s[2 * h + 1] - mu);
      l += p0 + p1;
      const float w0 = p0 * vs[2 * h], w1 = p1 * vs[2 * h + 1];
      psum += w0 + w1;
      const auto hi = __builtin_amdgcn_cvt_pkrtz(w0, w1);
      const auto lo = __builtin_amdgcn_cvt_pkrtz(w0 - (float)hi[0], w1 - (float)hi[1]);
      phi[h] = __builtin_bit_cast(uint32_t, hi);
      plo[h] = __builtin_bit_cast(uint32_t, lo);
    }
    const f16x8 pb_hi = __builtin_bit_cast(f16x8, u32x4{phi[0], phi[1], phi[2], phi[3]});
    const f16x8 pb_lo = __builtin_bit_cast(f16x8, u32x4{plo[0], plo[1], plo[2], plo[3]});
    // ---- O^T += V^T . P: tile mt takes nibble mt % 3 of codeword mt / 3
    uint32_t sv[8][VC];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (PACKED) {  // codeword c at byte vsh + 3c of the 12 loaded (alignbyte uses shift & 3)
        const uint32_t d0 = vw[j][0], d1 = vw[j][1], d2 = vw[j][2];
        vw[j][0] = __builtin_amdgcn_alignbyte(d1, d0, vsh);
        vw[j][1] = __builtin_amdgcn_alignbyte(vsh ? d2 : d1, vsh ? d1 : d0, vsh + 3);
        vw[j][2] = __builtin_amdgcn_alignbyte(d2, vsh < 2 ? d1 : d2, vsh + 2);
      }
#pragma unroll
      for (int c = 0; c < VC; ++c) sv[j][c] = sp_of(vw[j][c]);
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      uint32_t p[4];
#pragma unroll
      for (int h = 0; h < 4; ++h) p[h] = pair(sv[2 * h + 1][mt / 3], sv[2 * h][mt / 3], mt % 3, mt % 3);
      const f16x8 va = __builtin_bit_cast(f16x8, u32x4{p[0], p[1], p[2], p[3]});
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb_hi, acc[mt], 0, 0, 0);
      acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(va, pb_lo, acc[mt], 0, 0, 0);
    }
  }

  // ---- merge, as in the H(8,4) kernel
  l += __shfl_xor(l, 16, kWave);
  l += __shfl_xor(l, 32, kWave);
  psum += __shfl_xor(psum, 16, kWave);
  psum += __shfl_xor(psum, 32, kWave);
  const float poff = kOff * psum;
  if (n < G) {
    if (g == 0) {
      gml[0][wave][n] = m;
      gml[1][wave][n] = l;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int d = MT * (4 * g + r) + mt;
        if (d < D) red[wave][n][d] = acc[mt][r] * kScale - poff;
      }
  }
  __syncthreads();
  const int64_t ws_stride = a.nsplit * (a.d + 2);
  float *ws0 = a.ws + ((b * a.heads + h0) * a.nsplit + blockIdx.x) * (a.d + 2);
  for (int idx = threadIdx.x; idx < G * D; idx += kBlock) {
    const int h = idx / D, d = idx % D;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) M = fmaxf(M, gml[0][w][h]);
    float o = 0.0f, L = 0.0f;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) {
      const float mw = gml[0][w][h];
      const float wt = mw == -INFINITY ? 0.0f : attn_exp(mw - M);
      o += red[w][h][d] * wt;
      L += gml[1][w][h] * wt;
    }
    float *ws = ws0 + h * ws_stride;
    ws_put(ws + 2 + d, o);
    if (d == 0) {
      ws_put(ws, M);
      ws_put(ws + 1, L);
    }
  }
  if (a.ctr) combine_if_last<__half, G>(a, b * a.heads + h0, reinterpret_cast<float *>(rows));
}

template <typename T>
static void launch_combine(const AttnArgs &a, int64_t batch, hipStream_t st) {
  if (a.nsplit <= kCombineWaveSplits && a.d <= 2 * kWave)
    KVECC_LAUNCH(paged_attn_combine_wave_kernel<T>, dim3((unsigned)(batch * a.heads)), dim3(2 * kWave), 0, st, a);
  else
    KVECC_LAUNCH(paged_attn_combine_kernel<T>, dim3((unsigned)(batch * a.heads)), dim3(kBlock), 0, st, a);
}

static int pow2_at_least(int64_t x) {
  int w = 1;
  while (w < x) w <<= 1;
  return w;
}

template <typename T, int CODEC, int VEC, bool BUF>
static int launch_split_w(const AttnArgs &a, dim3 grid, hipStream_t st) {
  const int w = pow2_at_least((a.g + VEC - 1) / VEC);
  switch (w) {
#define KVECC_ATTN_CASE(WW)                                                                       \
  case WW:                                                                                        \
    KVECC_LAUNCH((paged_attn_split_kernel<T, CODEC, VEC, WW, BUF, 1>), grid, dim3(kBlock), 0, st, a); \
    return KVECC_OK;
    KVECC_ATTN_CASE(1)
    KVECC_ATTN_CASE(2)
    KVECC_ATTN_CASE(4)
    KVECC_ATTN_CASE(8)
    KVECC_ATTN_CASE(16)
    KVECC_ATTN_CASE(32)
    KVECC_ATTN_CASE(64)
#undef KVECC_ATTN_CASE
    default:
      return set_error(KVECC_EINVAL, "paged_attention: %lld lane chunks per token row > 64",
                       (long long)((a.g + VEC - 1) / VEC));
  }
}

template <typename T, int CODEC, int VEC>
static int launch_split(const AttnArgs &a, dim3 grid, hipStream_t st) {
  return a.cache_bytes ? launch_split_w<T, CODEC, VEC, true>(a, grid, st)
                       : launch_split_w<T, CODEC, VEC, false>(a, grid, st);
}

// words per lane of a token row: the VEC the codec's kernels use at head_dim d
// (the H(8,4) GQA kernels take 2 words = 8 codewords per lane: with G query
// rows and accumulators per lane, 4 words took 188 VGPRs at G = 4)
constexpr int kH84GqaVec = 2;
static int attn_vec(int codec, int64_t d, bool gqa = false) {
  if (codec == KVECC_CODEC_H84)
    return gqa && d % 8 == 0 ? kH84GqaVec : d % (4 * kH84Vec) == 0 ? kH84Vec : d % 16 == 0 ? 4 : 1;
  return codec == KVECC_CODEC_GOLAY ? kGolayVec : kGolayPackedVec;
}

// query heads per workgroup: the GQA kernels cover buffer-addressed caches with
// lane groups of 8-32 lanes per row (head_dim 64-256) and G in {2, 4} dividing
// H / Hkv (G 8 would hold 8 query rows and accumulators per lane); else 1
static int attn_heads_per_wg(int codec, int64_t d, int64_t g, int64_t heads, int64_t kv_heads, bool buf) {
  const int64_t group = heads / kv_heads;
  const int vec = attn_vec(codec, d, true);
  const int w = pow2_at_least((g + vec - 1) / vec);
  if (!buf || w < 8 || w > 32 || (codec == KVECC_CODEC_H84 && d % 8 != 0)) return 1;
  const int gmax = codec == KVECC_CODEC_GOLAY_PACKED ? 2 : 4;  // packed: G = 2 (the realigned loads' registers)
  return group % 4 == 0 && gmax >= 4 ? 4 : group % 2 == 0 ? 2 : 1;
}

template <typename T, int CODEC, int VEC, int G>
static int launch_split_gqa(const AttnArgs &a, dim3 grid, hipStream_t st) {
  switch (pow2_at_least((a.g + VEC - 1) / VEC)) {
    case 8: KVECC_LAUNCH((paged_attn_split_kernel<T, CODEC, VEC, 8, true, G>), grid, dim3(kBlock), 0, st, a); break;
    case 16: KVECC_LAUNCH((paged_attn_split_kernel<T, CODEC, VEC, 16, true, G>), grid, dim3(kBlock), 0, st, a); break;
    default: KVECC_LAUNCH((paged_attn_split_kernel<T, CODEC, VEC, 32, true, G>), grid, dim3(kBlock), 0, st, a); break;
  }
  return KVECC_OK;
}

template <typename T, int CODEC, int VEC>
static int launch_split_g(const AttnArgs &a, int64_t batch, int gq, hipStream_t st) {
  dim3 grid((unsigned)a.nsplit, (unsigned)(batch * a.heads / gq));
  if (gq == 1) return launch_split<T, CODEC, VEC>(a, grid, st);
  constexpr int GV = CODEC == KVECC_CODEC_H84 ? kH84GqaVec : VEC;
  if constexpr (CODEC != KVECC_CODEC_GOLAY_PACKED)
    if (gq == 4) return launch_split_gqa<T, CODEC, GV, 4>(a, grid, st);
  return launch_split_gqa<T, CODEC, GV, 2>(a, grid, st);
}

template <typename T, int CODEC>
static int launch_attn(const AttnArgs &a, int64_t batch, int gq, hipStream_t st) {
  int rc;
  if constexpr (CODEC == KVECC_CODEC_H84) {
    if (a.d % (4 * kH84Vec) == 0)
      rc = launch_split_g<T, CODEC, kH84Vec>(a, batch, gq, st);  // 16-byte loads, 16 codewords per lane
    else if (a.d % 16 == 0)
      rc = launch_split_g<T, CODEC, 4>(a, batch, gq, st);
    else
      rc = launch_split_g<T, CODEC, 1>(a, batch, gq, st);
  } else if constexpr (CODEC == KVECC_CODEC_GOLAY) {
    rc = launch_split_g<T, CODEC, kGolayVec>(a, batch, gq, st);  // 3 codewords per lane: 43 -> 15 of 16 lanes
  } else {
    rc = launch_split_g<T, CODEC, kGolayPackedVec>(a, batch, gq, st);  // 3 codewords per lane: 43 -> 15 of 16
  }
  if (rc != KVECC_OK) return rc;
  if (!a.ctr) launch_combine<T>(a, batch, st);
  return KVECC_OK;
}

template <int D>
static int launch_mfma_d(const AttnArgs &a, int64_t batch, int gm, hipStream_t st) {
  const dim3 grid((unsigned)a.nsplit, (unsigned)(batch * a.heads / gm));
  switch (gm) {
    case 1: KVECC_LAUNCH((paged_attn_h84_mfma_kernel<D, 1>), grid, dim3(kBlock), 0, st, a); break;
    case 2: KVECC_LAUNCH((paged_attn_h84_mfma_kernel<D, 2>), grid, dim3(kBlock), 0, st, a); break;
    case 4: KVECC_LAUNCH((paged_attn_h84_mfma_kernel<D, 4>), grid, dim3(kBlock), 0, st, a); break;
    case 8: KVECC_LAUNCH((paged_attn_h84_mfma_kernel<D, 8>), grid, dim3(kBlock), 0, st, a); break;
    default: KVECC_LAUNCH((paged_attn_h84_mfma_kernel<D, 16>), grid, dim3(kBlock), 0, st, a); break;
  }
  if (!a.ctr) launch_combine<__half>(a, batch, st);
  return KVECC_OK;
}

template <bool PACKED>
static int launch_golay_mfma(const AttnArgs &a, int64_t batch, int gm, hipStream_t st) {
  const dim3 grid((unsigned)a.nsplit, (unsigned)(batch * a.heads / gm));
  switch (gm) {
    case 2: KVECC_LAUNCH((paged_attn_golay_mfma_kernel<2, PACKED>), grid, dim3(kBlock), 0, st, a); break;
    case 4: KVECC_LAUNCH((paged_attn_golay_mfma_kernel<4, PACKED>), grid, dim3(kBlock), 0, st, a); break;
    case 8: KVECC_LAUNCH((paged_attn_golay_mfma_kernel<8, PACKED>), grid, dim3(kBlock), 0, st, a); break;
    default: KVECC_LAUNCH((paged_attn_golay_mfma_kernel<16, PACKED>), grid, dim3(kBlock), 0, st, a); break;
  }
  if (!a.ctr) launch_combine<__half>(a, batch, st);
  return KVECC_OK;
}

static int launch_mfma(int codec, const AttnArgs &a, int64_t batch, int gm, hipStream_t st) {
  if (codec != KVECC_CODEC_H84) {  // Golay, head_dim 128 (attn_mfma_heads)
    if (codec == KVECC_CODEC_GOLAY_PACKED) return launch_golay_mfma<true>(a, batch, gm, st);
    return launch_golay_mfma<false>(a, batch, gm, st);
  }
  switch (a.d) {
    case 32: return launch_mfma_d<32>(a, batch, gm, st);
    case 64: return launch_mfma_d<64>(a, batch, gm, st);
    default: return launch_mfma_d<128>(a, batch, gm, st);
  }
}

// query heads per workgroup of the MFMA kernels (0: not applicable): caches under
// 4 GiB, fp16 queries (16-byte aligned); Hamming(8,4) at head_dim 32 / 64 / 128
// for any group, Golay (int32 or packed) at head_dim 128 for groups of >= 2
// workgroups per CU of the Golay kernel's split choice (157 VGPRs, 49-73 KiB of
// LDS): 2 measured 30.6 vs 34.2 us at 4 (32q/8kv; profiles/r03/attn/attn_gqa14.log)
constexpr int kMfmaGolayWgPerCu = 2;
static int attn_mfma_heads(int codec, int q_dtype, const void *query, int64_t d, int64_t heads,
                           int64_t kv_heads, bool buf) {
  const int64_t group = heads / kv_heads;
  const bool h84 = codec == KVECC_CODEC_H84 && (d == 32 || d == 64 || d == 128);
  const bool golay = (codec == KVECC_CODEC_GOLAY || codec == KVECC_CODEC_GOLAY_PACKED) &&
                     d == 128;
  if (!(h84 || golay) || q_dtype != KVECC_F16 || !buf || !aligned(query, 16)) return 0;
  // MHA (one query head per cache head): H(8,4) too, one of the 16 MFMA
  // columns used -- the matrix cores take the dot products and the V update
  // off the VALU, and the table lookups are the only per-value LDS work:
  // [8,4096,32,128] 49.5 us per call against 54.6 for the VALU split kernel.
  // Golay MHA stays on the VALU kernels (packed 76 vs 68 us, int32 86 vs 73:
  // its per-codeword decode, not the arithmetic, is the work).
  // (tools/exp/run_attn_exp.py, profiles/r04/attn/mfma_mha_ab.log)
  if (group == 1) return h84 ? 1 : 0;
  return group % 16 == 0 ? 16 : group % 8 == 0 ? 8 : group % 4 == 0 ? 4 : group % 2 == 0 ? 2 : 0;
}

template <typename T>
static int launch_codec(int codec, const AttnArgs &a, int64_t batch, int gq, hipStream_t st) {
  switch (codec) {
    case KVECC_CODEC_H84: return launch_attn<T, KVECC_CODEC_H84>(a, batch, gq, st);
    case KVECC_CODEC_GOLAY: return launch_attn<T, KVECC_CODEC_GOLAY>(a, batch, gq, st);
    default: return launch_attn<T, KVECC_CODEC_GOLAY_PACKED>(a, batch, gq, st);
  }
}

// tokens per workgroup: the largest power of two <= kMaxSplit that still gives
// >= per_cu workgroups per CU (small batch*heads decode steps split finer); 8
// per CU made every codec 1-15 % slower
static int64_t choose_split(int64_t bh, int64_t max_context_len, int per_cu = 4) {
  // longer splits amortise each workgroup's fixed work (table staging, the
  // group merge); measured best at 1024 for both codecs at [8,4096,32,128]
  const int64_t top = kMaxSplit;
  int64_t split = top;
  const int64_t want = (int64_t)per_cu * cu_count();
  while (split > 32 && bh * cdiv(max_context_len, split) < want) split >>= 1;
  while (cdiv(max_context_len, split) > kMaxSplits && split < top) split <<= 1;
  return split;
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API int64_t kvecc_paged_attention_workspace(int64_t batch, int64_t heads, int64_t head_dim,
                                                  int64_t max_context_len) {
  if (batch <= 0 || heads <= 0 || head_dim <= 0 || max_context_len <= 0) return 0;
  // the GQA kernels split finer (their grid has H/G workgroups per split):
  // room for the finest, G = 4 (choose_split is monotone in its first argument)
  const int64_t bh = std::max<int64_t>(1, batch * heads / 4);
  return batch * heads * cdiv(max_context_len, choose_split(bh, max_context_len)) * (head_dim + 2);
}

KVECC_API int kvecc_paged_attention(const void *query, int q_dtype, const void *k_cache,
                                    const void *v_cache, const int32_t *block_table,
                                    const int32_t *context_lens, const float *k_scales,
                                    const float *v_scales, void *out, int64_t batch,
                                    int64_t heads, int64_t kv_heads, int64_t head_dim,
                                    int64_t num_blocks, int64_t num_layers, int64_t layer, int64_t block_size,
                                    int64_t max_blocks, int64_t max_context_len, float sm_scale,
                                    int codec, float *workspace, int64_t workspace_floats,
                                    void *stream) {
  if (batch < 0 || heads < 0 || kv_heads < 0 || head_dim < 0)
    return set_error(KVECC_EINVAL, "paged_attention: negative size");
  if (batch == 0 || heads == 0) return KVECC_OK;
  if (kv_heads < 1 || heads % kv_heads != 0)
    return set_error(KVECC_EINVAL, "paged_attention: %lld heads not a multiple of %lld kv heads",
                     (long long)heads, (long long)kv_heads);
  if (head_dim < 1 || head_dim > kAttnMaxD)
    return set_error(KVECC_EINVAL, "paged_attention: head_dim %lld not in [1, %d]", (long long)head_dim, kAttnMaxD);
  if (codec != KVECC_CODEC_H84 && codec != KVECC_CODEC_GOLAY && codec != KVECC_CODEC_GOLAY_PACKED)
    return set_error(KVECC_EINVAL, "paged_attention: codec %d (hamming84 or golay only)", codec);
  if (codec == KVECC_CODEC_H84 && head_dim % 4 != 0)
    return set_error(KVECC_EINVAL, "paged_attention: hamming84 head_dim must be a multiple of 4");
  if (num_layers < 1 || layer < 0 || layer >= num_layers || block_size < 1 || max_blocks < 1)
    return set_error(KVECC_EINVAL, "paged_attention: bad cache geometry");
  if (num_blocks < 1 || num_blocks * num_layers * kv_heads * block_size > 0x7FFFFFFFLL)
    return set_error(KVECC_EINVAL, "paged_attention: cache rows must fit int32");
  if (max_context_len <= 0) max_context_len = max_blocks * block_size;
  if (!query || !k_cache || !v_cache || !block_table || !context_lens || !k_scales || !v_scales ||
      !out || !workspace)
    return set_error(KVECC_EINVAL, "paged_attention: null pointer");
  const int64_t need = kvecc_paged_attention_workspace(batch, heads, head_dim, max_context_len);
  if (workspace_floats < need)
    return set_error(KVECC_EINVAL, "paged_attention: workspace %lld < %lld floats",
                     (long long)workspace_floats, (long long)need);
  AttnArgs a;
  a.q = query;
  a.k_cache = k_cache;
  a.v_cache = v_cache;
  a.table = block_table;
  a.ctx_lens = context_lens;
  a.k_scales = k_scales;
  a.v_scales = v_scales;
  a.ws = workspace;
  a.out = out;
  a.heads = heads;
  a.kv_heads = kv_heads;
  a.d = head_dim;
  a.g = codec == KVECC_CODEC_H84 ? head_dim / 4 : (head_dim + 2) / 3;
  a.rowb = (uint32_t)KVECC_GOLAY_PACKED_ROW(a.g);
  a.layers = num_layers;
  a.layer = layer;
  a.bs = block_size;
  a.max_blocks = max_blocks;
  a.sm_scale = sm_scale;
  a.empty_value = codec == KVECC_CODEC_H84 ? -8.0f : 0.0f;
  int gq = 1, gm = 0;
  {
    const int64_t rows_total = num_blocks * num_layers * kv_heads * block_size;
    const int64_t cb = rows_total * (codec == KVECC_CODEC_H84            ? head_dim
                                     : codec == KVECC_CODEC_GOLAY_PACKED ? (int64_t)a.rowb
                                                                         : 4 * a.g);
    const bool fits = cb <= 0xFFFFFFFFLL && rows_total * 4 <= 0xFFFFFFFFLL;
    a.cache_bytes = fits ? (uint32_t)cb : 0u;  // 0 selects the 64-bit-addressed kernels
    a.scale_bytes = fits ? (uint32_t)(rows_total * 4) : 0u;
    gq = attn_heads_per_wg(codec, head_dim, a.g, heads, kv_heads, fits);
    gm = attn_mfma_heads(codec, q_dtype, query, head_dim, heads, kv_heads, fits);
  }
  if (gm)  // kMfma*WgPerCu workgroups per CU, never finer than the workspace allows
    a.split = std::max(choose_split(batch * heads / gm, max_context_len,
                                    codec != KVECC_CODEC_H84 ? kMfmaGolayWgPerCu : kMfmaWgPerCu),
                       choose_split(std::max<int64_t>(1, batch * heads / 4), max_context_len));
  else
    a.split = choose_split(batch * heads / gq, max_context_len);
  a.nsplit = cdiv(max_context_len, a.split);
  if (a.nsplit > kMaxSplits)
    return set_error(KVECC_EINVAL, "paged_attention: context %lld too long", (long long)max_context_len);
  a.par = a.cor = nullptr;
  a.atab = a.atab_x = nullptr;
  a.ctr = nullptr;
  // fused combine for one query head per workgroup only (MHA 59.7 -> 58.9 us).
  // With G heads the tail after the last split -- the sc1 stores' acknowledgement,
  // the counter's round trip and rounds of sc1 loads, which bypass the L2 -- cost
  // more than the combine launch: 32q/8kv 22.6 -> 32.8 us with the G heads
  // combined serially, 26.9 with one wave per head, 26.7 (against 22.3) with all
  // G heads in one round trip (combine_group; profiles/r03/attn/).
  const int gw = gm ? gm : gq;  // query heads per workgroup
  if (gw == 1 && batch * heads <= kAttnCtrPerSlot) {
    a.ctr = attn_counter_slot(stream);
    if (!a.ctr) return KVECC_EHIP;
  }
  if (codec != KVECC_CODEC_H84) {
    a.par = golay_parity_table_dev();
    a.cor = golay_correct_table_dev();
    a.atab = golay_attn_table_dev();
    a.atab_x = golay_attn_x_table_dev();
    if (!a.par || !a.cor || !a.atab || !a.atab_x) return KVECC_EHIP;
  }
  hipStream_t st = as_stream(stream);
  if (gm) {
    const int rc = launch_mfma(codec, a, batch, gm, st);
    if (rc != KVECC_OK) return rc;
    return check_launch("paged_attention");
  }
  int rc;
  switch (q_dtype) {
    case KVECC_F32: rc = launch_codec<float>(codec, a, batch, gq, st); break;
    case KVECC_F16: rc = launch_codec<__half>(codec, a, batch, gq, st); break;
    case KVECC_BF16: rc = launch_codec<__hip_bfloat16>(codec, a, batch, gq, st); break;
    default: return set_error(KVECC_EINVAL, "paged_attention: bad dtype %d", q_dtype);
  }
  if (rc != KVECC_OK) return rc;
  return check_launch("paged_attention");
}

}  // extern "C"
