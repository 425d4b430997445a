/*
 * kvecc.h -- C ABI of the MI355X-native ECC KV-cache codec (libkvecc.so).
 *
 * This is the drop-in boundary for the reference's hot path,
 * ecc_codecs/triton_kernels/ (Hamming(7,4)/(8,4), Golay(24,12), Bernoulli bit
 * flip injection, double-error interpolation, fused quantize/encode and
 * decode/dequantize).  The reference exposes these as Python functions over
 * torch tensors; each entry point below replaces the Triton kernel + wrapper
 * cited next to it (paths relative to the reference repository root).  The
 * Python host package `kvecc` binds them with ctypes.
 *
 * Conventions (all entry points):
 *   - Pointers are DEVICE pointers (hipMalloc / torch CUDA tensors) unless the
 *     name ends in _host.  Buffers must not overlap unless stated.
 *   - `stream` is a hipStream_t (NULL = legacy default stream).  Calls only
 *     enqueue work: no allocation, no host synchronisation (graph-capturable
 *     once kvecc_init_device() has run for the device).
 *   - Statistics accumulate (+=) into a caller-provided, zero-initialised device
 *     buffer of KVECC_STATS_WORDS uint64 words, or are skipped when the pointer
 *     is NULL.  The buffer is sharded: workgroup g adds its partial sums to
 *     slot (g % KVECC_STATS_SLOTS), one 128-byte line per slot, and statistic k
 *     (the "stats[k]" named below) is  sum over s of buf[s*KVECC_STATS_STRIDE + k].
 *     (Thousands of device-scope atomics on ONE address serialise at ~10 ns
 *     each -- longer than the kernels themselves.)
 *   - Return 0 on success, a negative KVECC_E* code on failure; the message is
 *     available from kvecc_last_error() (thread-local).
 *   - n / m / rows == 0 is valid and enqueues nothing.
 */
#ifndef KVECC_H
#define KVECC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KVECC_API __attribute__((visibility("default")))

enum {
  KVECC_OK = 0,
  KVECC_EINVAL = -1, /* bad argument (null pointer, negative size, bad enum) */
  KVECC_EHIP = -2,   /* HIP runtime error (launch / memory)                  */
  KVECC_ENODEV = -3  /* no HIP device                                         */
};

/* statistics buffer geometry (see conventions above) */
#define KVECC_STATS_SLOTS 32
#define KVECC_STATS_STRIDE 16 /* uint64 words per slot = one 128-B line */
#define KVECC_STATS_WORDS (KVECC_STATS_SLOTS * KVECC_STATS_STRIDE)

/* dtype codes for fused kernels */
enum { KVECC_F32 = 0, KVECC_F16 = 1, KVECC_BF16 = 2 };
/* codec codes for fused kernels */
enum { KVECC_CODEC_NONE = 0, KVECC_CODEC_H74 = 1, KVECC_CODEC_H84 = 2, KVECC_CODEC_GOLAY = 3,
       /* shim caches only (kvecc_shim_write / kvecc_shim_read and the cpu twins):
        * Golay(24,12) codewords stored as 3 little-endian bytes, a token row of
        * g = ceil(d/3) codewords padded to KVECC_GOLAY_PACKED_ROW(g) bytes --
        * 132 B instead of the reference's 172 B (int32) at d = 128 */
       KVECC_CODEC_GOLAY_PACKED = 4 };
#define KVECC_GOLAY_PACKED_ROW(g) ((3 * (g) + 3) / 4 * 4)

/* Row scale rule of the INT4 quantizer.  The reference computes
 * `abs_max / 7.0` with a Python-scalar divisor (paged_cache_ecc.py:330); torch
 * evaluates that as IEEE division on CPU tensors but as abs_max * RN(1/7) on
 * GPU tensors (its CPU-scalar-divisor shortcut), and the two differ in ~55% of
 * rows.  DIV7 reproduces the reference run on the CPU (the golden fixtures),
 * MUL_INV7 the reference run on a GPU.  q = x / scale is IEEE under both. */
enum { KVECC_SCALE_DIV7 = 0, KVECC_SCALE_MUL_INV7 = 1 };

/* ---- runtime --------------------------------------------------------------- */
KVECC_API const char *kvecc_version(void);
KVECC_API const char *kvecc_last_error(void);
KVECC_API int kvecc_device_count(void);
/* Kernel timing without marker packets: the NEXT kernel this thread launches
 * through any kvecc_* device entry point records its own start and end into
 * the given hipEvent_t's (either may be NULL) via hipExtLaunchKernel, then the
 * hook disarms.  Entry points that launch a main kernel and a tail kernel time
 * the first one.  The reference has no counterpart (benchmark_harness.py:42-57
 * brackets launches with events); bench.py uses this to time every step. */
KVECC_API int kvecc_time_next_launch(void *start_event, void *stop_event);
/* Upload the Golay tables to `device` (done lazily otherwise; call before graph
 * capture).  Replaces golay_triton.py:304-330 (_build_syndrome_table cache). */
KVECC_API int kvecc_init_device(int device);
/* Work / split counters of the dynamically scheduled kernels (the fused shim
 * reads, the per-head Golay rows, the packed decodes, the paged-attention fused
 * combine).  No reference counterpart: the reference launches one program per
 * row and schedules nothing.  Each kernel needs its counters zero and to itself
 * while it runs, and leaves them zero.  The library gives eager launches one
 * counter slot per stream (per thread for hipStreamPerThread; keyed by the
 * stream's address -- a stream created at a destroyed stream's address inherits
 * its slot, safe because hipStreamDestroy drains the queue first), and
 * launches captured into a graph a slot of their own per (capture, stream), so
 * launches that can overlap never share counters.  Slots (48 KiB each) come
 * from a pool that grows from eager launches only (never inside the launching
 * stream's own capture): every eager launch of such a kernel tops the free list
 * back up to 32 slots, so 32 captures can follow any eager launch;
 * kvecc_reserve_counter_slots(device, n) makes n more available ahead of a
 * longer run of captures.  Growth allocates in relaxed capture mode, so an
 * eager launch beside another stream's global-mode capture (torch.cuda.graph's
 * default) neither fails nor invalidates that capture.  A captured slot is tied to its graph by
 * a HIP user object and returns to the pool when the graph and all its
 * executable instances are destroyed.  A graph keeps its slots for every
 * replay: replay one graph on one stream at a time (two overlapping replays of
 * the same graph would share counters). */
KVECC_API int kvecc_reserve_counter_slots(int device, int n);
/* Diagnostic (synchronises the device): slots handed out, and how many counter
 * words of all slots are non-zero -- 0 whenever no launch is in flight. */
KVECC_API int kvecc_counter_slots_check(int device, int64_t *slots_in_use, int64_t *nonzero_words);
/* Test hook: on != 0 makes the step that ties a captured launch's slot to its
 * graph fail (as hipGraphRetainUserObject might); such a slot then stays with
 * its capture for the life of the process instead of returning to the pool. */
KVECC_API int kvecc_debug_fail_graph_retain(int on);
/* Host copies of the code tables the kernels use (for verification):
 *   syndrome table as the reference builds it, config.py:403-457 -> int32[4096]
 *   H row masks, config.py:354-379 -> uint32[12]                              */
KVECC_API int kvecc_golay_syndrome_table_host(int32_t *out4096);
KVECC_API int kvecc_golay_h_row_masks_host(uint32_t *out12);
/* Integer form of the reference's `tl.rand(..) < ber` test (random.py:126-143):
 * the smallest folded 31-bit value x with fp32(x)*0x2FFFFFFF >= fp32(ber). */
KVECC_API uint32_t kvecc_ber_threshold(float ber);

/* ---- Hamming(7,4) / Hamming(8,4) ------------------------------------------ */
/* hamming74_triton.py:48-91 + :170-201 */
KVECC_API int kvecc_hamming74_encode(const uint8_t *in, uint8_t *out, int64_t n, void *stream);
/* hamming74_triton.py:100-162 + :218-277 ; stats[0] += #syndrome != 0 */
KVECC_API int kvecc_hamming74_decode(const uint8_t *cw, uint8_t *data, uint8_t *flag,
                                     int64_t n, uint64_t *stats, void *stream);
/* hamming84_triton.py:50-108 + :217-254 */
KVECC_API int kvecc_hamming84_encode(const uint8_t *in, uint8_t *out, int64_t n, void *stream);
/* hamming84_triton.py:117-209 + :281-351 ; error_type may be NULL;
 * stats[0] += #SINGLE_CORRECTED, stats[1] += #DOUBLE_DETECTED */
KVECC_API int kvecc_hamming84_decode(const uint8_t *cw, uint8_t *data, uint8_t *error_type,
                                     int64_t n, uint64_t *stats, void *stream);

/* ---- Golay(24,12) ------------------------------------------------------------ */
/* golay_triton.py:99-157 + :382-422 ; triplets uint8[m][3] -> int32[m] */
KVECC_API int kvecc_golay_encode(const uint8_t *triplets, int32_t *codewords, int64_t m,
                                 void *stream);
/* golay_triton.py:213-295 + :425-498 ; counts may be NULL;
 * stats[0] += sum of counts < 4 (bits corrected), stats[1] += #count == 4 */
KVECC_API int kvecc_golay_decode(const int32_t *codewords, uint8_t *triplets, uint8_t *counts,
                                 int64_t m, uint64_t *stats, void *stream);
/* Per-head packing of the shim (ecc_shim.py:623-624,669-682): each row of d
 * nibbles is zero-padded to 3*ceil(d/3) and encoded to ceil(d/3) codewords. */
KVECC_API int kvecc_golay_encode_rows(const uint8_t *nibbles, int32_t *codewords, int64_t rows,
                                      int64_t d, void *stream);
/* Inverse of the above (ecc_shim.py:990-1008): decoded rows of d nibbles. */
KVECC_API int kvecc_golay_decode_rows(const int32_t *codewords, uint8_t *nibbles,
                                      int64_t rows, int64_t d, uint64_t *stats, void *stream);

/* ---- Bernoulli bit-flip injection ------------------------------------------- */
/* fault_injection_triton.py:228-299 (uint8) and :303-334 (int32), wrapper
 * :337-424.  Element i is global element offset0+i of a global_n-element flat
 * tensor (pass global_n = n, offset0 = 0 for the unsharded call), so shards
 * reproduce the single-device flip pattern.  counts (uint8 per element) may be
 * NULL; stats[0] += flips, stats[1] += elements with >=1 flip.  in == out is
 * allowed (in-place). */
KVECC_API int kvecc_inject_u8(const uint8_t *in, uint8_t *out, uint8_t *counts, int64_t n,
                              int n_bits, int64_t seed, float ber, int64_t global_n,
                              int64_t offset0, uint64_t *stats, void *stream);
KVECC_API int kvecc_inject_i32(const int32_t *in, int32_t *out, uint8_t *counts, int64_t n,
                               int n_bits, int64_t seed, float ber, int64_t global_n,
                               int64_t offset0, uint64_t *stats, void *stream);
/* rand4x variants, fault_injection_triton.py:57-133 / :137-224 / :434-496 */
KVECC_API int kvecc_inject_u8_vectorized(const uint8_t *in, uint8_t *out, uint8_t *counts,
                                         int64_t n, int n_bits, int64_t seed, float ber,
                                         uint64_t *stats, void *stream);
KVECC_API int kvecc_inject_i32_vectorized(const int32_t *in, int32_t *out, uint8_t *counts,
                                          int64_t n, int n_bits, int64_t seed, float ber,
                                          uint64_t *stats, void *stream);
/* Per-row scheme of the shim (ecc_shim.py:643-651,684-691,713-721): row r
 * (row_len elements, contiguous, rows back to back) is injected as its own
 * call with N = row_len and seed = seed_base + r.  in == out allowed. */
KVECC_API int kvecc_inject_rows_u8(const uint8_t *in, uint8_t *out, int64_t rows,
                                   int64_t row_len, int n_bits, int64_t seed_base, float ber,
                                   uint64_t *stats, void *stream);
KVECC_API int kvecc_inject_rows_i32(const int32_t *in, int32_t *out, int64_t rows,
                                    int64_t row_len, int n_bits, int64_t seed_base, float ber,
                                    uint64_t *stats, void *stream);

/* ---- Interpolation ----------------------------------------------------------- */
/* interpolation_triton.py:120-159 + :162-265 on a contiguous [outer][len][inner]
 * uint8 array whose sequence axis is the middle one (no permute copies).
 * err == 2 elements become round_half_up((q[l-1]+q[l+1])/2) from clamped
 * neighbours, every element is clamped to [0,15] -- unless `gate` is non-NULL
 * and *gate == 0 (device int32), in which case out = q (the reference's
 * no-double fast path, :199-201, decided on the device). */
KVECC_API int kvecc_interpolate(const uint8_t *q, const uint8_t *err, uint8_t *out,
                                int64_t outer, int64_t len, int64_t inner, const int32_t *gate,
                                void *stream);
/* The reference wrapper in full (interpolation_triton.py:162-265) in one pass:
 * out = the interpolated, clamped result when any err == 2, else out = q (its
 * `q.clone()` fast path, :199-201).  No host sync, no separate scan of err and
 * no zeroing pass: the kernel sets flags[0] = epoch if any err == 2 and
 * flags[1] = epoch if any q > 15 (device int32[2]); a trailing copy kernel
 * restores out = q only when flags[0] != epoch and flags[1] == epoch (without
 * doubles, clamping is visible only where q > 15).  `epoch` must be non-zero
 * and differ from both words of `flags` on entry (e.g. a per-buffer call
 * counter); afterwards "flags[k] == epoch" reads as "condition k was seen". */
KVECC_API int kvecc_interpolate_auto(const uint8_t *q, const uint8_t *err, uint8_t *out,
                                     int64_t outer, int64_t len, int64_t inner, int32_t *flags,
                                     int32_t epoch, void *stream);
/* *flag = (any x[i] == value) ? 1 : 0 (device int32, overwritten). */
KVECC_API int kvecc_any_equal_u8(const uint8_t *x, int64_t n, uint8_t value, int32_t *flag,
                                 void *stream);
/* stats[0] += number of positions i < n with a[i] != b[i] (device buffers;
 * sharded statistics buffer as the codecs use).  The codec-level sweep's
 * residual-error count, `(decoded != truth).sum()` in the reference's Monte
 * Carlo (evaluation/experiments/monte_carlo.py:75-395), as one HBM pass. */
KVECC_API int kvecc_count_ne_u8(const uint8_t *a, const uint8_t *b, int64_t n, uint64_t *stats,
                                void *stream);

/* ---- Monte-Carlo trial (BASELINE config 5) ---------------------------------- */
/* One trial of the codec-level fault-injection sweep in one launch: for every
 * value of the ground-truth INT4 tensor x [outer, len, heads, head_dim] (uint8
 * nibbles, contiguous), encode -> Bernoulli flips (the reference's per-bit
 * Philox stream of fault_injection_triton.py:228-334 over the shard's global
 * indices: global_n elements, this shard starting at offset0) -> decode
 * (-> double-error interpolation along `len`) -> compare with x, keeping only
 * the statistics; the codewords and decoded values never reach HBM.  The
 * counterpart of the reference's encode / inject_bit_errors_triton / decode
 * trial (evaluation/experiments/quantization_ecc_comparison.py:164-203,
 * evaluation/sweep.py:352-626) and exactly the counters of that pipeline run
 * kernel by kernel:
 *   stats[0] flips, stats[1] elements with >= 1 flip,
 *   stats[2] corrected (H74: syndrome != 0; H84: single errors; Golay: bits),
 *   stats[3] detected (H74: 0; H84: double errors; Golay: uncorrectable words),
 *   stats[4] decoded (interpolated) values != x.
 * Hamming codecs draw n_bits 7 / 8 per value (global_n, offset0 in values);
 * Golay packs each head row into ceil(head_dim/3) codewords (the shim's
 * per-head padding, ecc_shim.py:623-682) and draws 24 bits per codeword
 * (global_n, offset0 in codewords).  KVECC_MC_H84_INTERP needs heads*head_dim
 * % 4 == 0. */
enum { KVECC_MC_H74 = 1, KVECC_MC_H84 = 2, KVECC_MC_H84_INTERP = 3, KVECC_MC_GOLAY = 4 };
KVECC_API int kvecc_mc_trial(const uint8_t *x, int64_t outer, int64_t len, int64_t heads,
                             int64_t head_dim, int codec, float ber, int64_t seed, int64_t global_n,
                             int64_t offset0, uint64_t *stats, void *stream);
/* dst[b * dst_stride + w] += stats word w summed over the KVECC_STATS_SLOTS
 * slots of buffer b (buffers KVECC_STATS_WORDS apart), for b < nbuf and
 * w < nwords <= KVECC_STATS_STRIDE; the buffers are zeroed afterwards.  One
 * launch folds every trial's counters into the sweep's table. */
KVECC_API int kvecc_stats_fold(uint64_t *stats, int64_t nbuf, int nwords, int64_t *dst,
                               int64_t dst_stride, void *stream);

/* ---- Fused quantize / encode and decode / dequantize ----------------------- */
/* fused_kernels.py:18-160 (H84), :163-269 (H74), and the shim's torch path
 * ecc_shim.py:572-580: per row of d values (dtype x_dtype), scale = absmax/7
 * under `scale_rule` (KVECC_SCALE_*; 0 -> 1), q = rint(x/scale) clamped [-8,7]
 * + 8, then encoded with `codec` (KVECC_CODEC_NONE stores the raw nibble).
 * scales: fp32 per row. */
KVECC_API int kvecc_quantize_encode_rows(const void *x, int x_dtype, int codec, int scale_rule,
                                         uint8_t *cw, float *scales, int64_t rows, int64_t d,
                                         void *stream);
/* fused_kernels.py:272-437 : H84 decode + (q-8)*scale -> out (out_dtype).
 * zero_doubles = 1 reproduces :344 (double-error data -> 0).
 * stats[0] += #SINGLE_CORRECTED, stats[1] += #DOUBLE_DETECTED. */
KVECC_API int kvecc_decode_dequant_h84_rows(const uint8_t *cw, const float *scales, void *out,
                                            int out_dtype, int64_t rows, int64_t d,
                                            int zero_doubles, uint64_t *stats, void *stream);

/* ---- Packed Golay storage (native layout, not the reference's) -- */
/* values as INT4 nibbles two per byte (value j in byte j/2, low nibble first),
 * codewords as 3 little-endian bytes (data12 | parity12 << 12, as
 * golay_triton.py:130-155), so codeword k covers values 3k..3k+2.
 * nibbles: ceil(3m/2) bytes; codewords: 3m bytes; uncorrectable (may be NULL):
 * ceil(m/8) bytes, bit k%8 of byte k/8 = codeword k uncorrectable (data kept);
 * stats[0] += bits corrected, stats[1] += #uncorrectable.  Decode moves 4.625 B
 * per codeword (reference layout: 8), encode 4.5 B (reference: 7). */
KVECC_API int kvecc_golay_encode_packed(const uint8_t *nibbles, uint8_t *codewords, int64_t m,
                                        void *stream);
KVECC_API int kvecc_golay_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                        uint8_t *uncorrectable, int64_t m, uint64_t *stats,
                                        void *stream);

/* Hamming(8,4) with packed values: nibbles two per byte (as above), codewords
 * one byte each (the reference's), error types 2 bits per value (value j at
 * bits 2*(j%4) of byte j/4; may be NULL).  stats as kvecc_hamming84_decode.
 * Encode moves 1.5 B/value (reference layout: 2), decode 1.75 (reference: 3). */
KVECC_API int kvecc_hamming84_encode_packed(const uint8_t *nibbles, uint8_t *codewords, int64_t n,
                                            void *stream);
KVECC_API int kvecc_hamming84_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                            uint8_t *error_types, int64_t n, uint64_t *stats,
                                            void *stream);

/* ---- ECC shim: KV-cache write and read -------------------------------------- */
/* ecc_shim.py:557-721 (ECCBackend.write) for codec KVECC_CODEC_NONE (int4),
 * H74, H84, GOLAY in ONE launch: K and V [batch, seq, hkv*d] (x_dtype,
 * contiguous) are quantized per (pos, head) row (absmax/7 under scale_rule,
 * round-half-even),
 * encoded, injected with the row's own seed when `inject` and ber > 0
 * (K: seed0 + r, V: seed0 + r + 1, r = (b*seq + pos)*hkv + h; n_bits per
 * codeword as ecc_shim.py:555-560) and stored into the paged caches -- only the
 * last batch, which is what the reference's same-slot writes leave behind.
 * Caches: [blocks, num_layers, hkv, block_size, P] with P = d (uint8) or
 * ceil(d/3) (int32, Golay per-head padding), or KVECC_GOLAY_PACKED_ROW(ceil(d/3))
 * bytes for KVECC_CODEC_GOLAY_PACKED (not a reference layout); scales fp32 [blocks, num_layers,
 * hkv, block_size]; token pos lives in physical block block_table[pos / block_size]
 * (device int32).  d <= 512. */
KVECC_API int kvecc_shim_write(const void *k, const void *v, int x_dtype, int64_t batch,
                               int64_t seq, int64_t hkv, int64_t d, int codec, int scale_rule,
                               int n_bits,
                               int inject, float ber, int64_t seed0, void *k_cache, void *v_cache,
                               float *k_scales, float *v_scales, const int32_t *block_table,
                               int64_t num_layers, int64_t block_size, int64_t layer,
                               void *stream);
/* kvecc_shim_write on strided K/V: element (b, pos, h, e) of K lives at
 * k[b*k_batch_stride + pos*k_seq_stride + h*k_head_stride + e] (same for V;
 * each head's d values contiguous), so the projections' views are read in
 * place -- a slice of GPT-2's fused c_attn output, or Llama's post-RoPE
 * [b, h, s, d] tensor transposed -- where the reference first copies them
 * with .transpose(1, 2).contiguous() (ecc_shim.py:1290-1291, :1351-1352).
 * Strides are >= 0 and head strides >= d. */
KVECC_API int kvecc_shim_write_strided(const void *k, const void *v, int64_t k_batch_stride,
                                       int64_t k_seq_stride, int64_t k_head_stride,
                                       int64_t v_batch_stride, int64_t v_seq_stride,
                                       int64_t v_head_stride, int x_dtype, int64_t batch,
                                       int64_t seq, int64_t hkv, int64_t d, int codec,
                                       int scale_rule, int n_bits, int inject, float ber,
                                       int64_t seed0, void *k_cache, void *v_cache,
                                       float *k_scales, float *v_scales,
                                       const int32_t *block_table, int64_t num_layers,
                                       int64_t block_size, int64_t layer, void *stream);
/* ecc_shim.py:990-1071 (ECCBackend.attend, decode side) in ONE launch: gather
 * the first ctx tokens of layer `layer`, decode (H74: stats[0] += #flagged;
 * H84: stats[0] += #SINGLE_CORRECTED, stats[1] += #DOUBLE_DETECTED; Golay:
 * stats[0] += bits corrected, stats[1] += #uncorrectable; stats may be NULL),
 * interpolate H84 double errors along the context when `interp`, dequantize
 * (q - 8) * scale in fp32 and store k_out / v_out as [hkv, ctx, d] in out_dtype
 * (RNE).  Byte codecs need d % 4 == 0. */
KVECC_API int kvecc_shim_read(const void *k_cache, const void *v_cache, const float *k_scales,
                              const float *v_scales, const int32_t *block_table, int64_t ctx,
                              int64_t hkv, int64_t d, int64_t num_layers, int64_t block_size,
                              int64_t layer, int codec, int interp, void *k_out, void *v_out,
                              int out_dtype, uint64_t *stats, void *stream);
/* kvecc_shim_read over `batch` sequences in one call: sequence b reads its first
 * ctx tokens through block_table row b (block_table[b * table_stride + lb],
 * table_stride >= ceil(ctx / block_size)); k_out / v_out are [batch, hkv, ctx,
 * d].  Golay caches with d % 8 == 0 take the wave-tile kernel (one launch for
 * every sequence and both sides; the fused decode BASELINE's north_star
 * measures); the other codecs launch once per sequence.  Every codec reads a
 * negative block id as zero codewords: its rows output +0 (no statistics), and
 * as an H84 interpolation neighbour its values read as decode(0) = 0.  batch 1
 * is kvecc_shim_read. */
KVECC_API int kvecc_shim_read_batch(const void *k_cache, const void *v_cache, const float *k_scales,
                                    const float *v_scales, const int32_t *block_table,
                                    int64_t table_stride, int64_t batch, int64_t ctx, int64_t hkv,
                                    int64_t d, int64_t num_layers, int64_t block_size, int64_t layer,
                                    int codec, int interp, void *k_out, void *v_out, int out_dtype,
                                    uint64_t *stats, void *stream);

/* ---- Paged decode attention with inline ECC decode ---------------------------- */
/* attention_ecc.py:620-780 (paged_attention_ecc) + :265-427 (kernel): one query
 * token per sequence, query [batch, heads, head_dim] (q_dtype), caches as above
 * (codec H84: uint8, double errors keep their data; GOLAY: int32, uncorrectable
 * data kept; GOLAY_PACKED: 3-byte codewords, rows of KVECC_GOLAY_PACKED_ROW bytes), block_table [batch, max_blocks] int32 (-1 = no block, token
 * skipped), context_lens [batch] int32 (<= max_context_len; <= 0 means
 * max_blocks*block_size), out [batch, heads, head_dim] in q_dtype.  A sequence
 * with no valid token (context_len <= 0 or only -1 blocks) gets the reference's
 * values: -8.0 in every lane for H84 (its kernel's -1e20 masking,
 * attention_ecc.py:342,391-423), 0 for Golay (reference_attention_ecc).  Query head h reads cache head h / (heads / kv_heads).  `workspace`:
 * kvecc_paged_attention_workspace(...) floats.  head_dim <= 256. */
KVECC_API int64_t kvecc_paged_attention_workspace(int64_t batch, int64_t heads, int64_t head_dim,
                                                  int64_t max_context_len);
KVECC_API int kvecc_paged_attention(const void *query, int q_dtype, const void *k_cache,
                                    const void *v_cache, const int32_t *block_table,
                                    const int32_t *context_lens, const float *k_scales,
                                    const float *v_scales, void *out, int64_t batch,
                                    int64_t heads, int64_t kv_heads, int64_t head_dim,
                                    int64_t num_blocks, int64_t num_layers, int64_t layer, int64_t block_size,
                                    int64_t max_blocks, int64_t max_context_len, float sm_scale,
                                    int codec, float *workspace, int64_t workspace_floats,
                                    void *stream);

/* ---- Host ("cpu") backend ------------------------------------------------- */
/* The reference has no CPU codec backend (every wrapper asserts x.is_cuda,
 * e.g. hamming74_triton.py:185,246, golay_triton.py:399,456); BASELINE config 1 asks
 * for backend="cpu".  These are the host twins of the entry points above:
 * same arguments minus the stream, HOST pointers, the same codec algebra
 * (csrc/codec_math.h) run by `threads` std::threads (<= 0: all cores).
 * `stats` is a plain host uint64 array (stats[0], stats[1] += ...), not the
 * sharded device buffer. */
KVECC_API int kvecc_cpu_hamming74_encode(const uint8_t *in, uint8_t *out, int64_t n, int threads);
KVECC_API int kvecc_cpu_hamming84_encode(const uint8_t *in, uint8_t *out, int64_t n, int threads);
KVECC_API int kvecc_cpu_hamming74_decode(const uint8_t *cw, uint8_t *data, uint8_t *flag, int64_t n,
                                         uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_hamming84_decode(const uint8_t *cw, uint8_t *data, uint8_t *etype, int64_t n,
                                         uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_golay_encode(const uint8_t *trip, int32_t *cw, int64_t m, int threads);
KVECC_API int kvecc_cpu_golay_decode(const int32_t *cw, uint8_t *trip, uint8_t *counts, int64_t m,
                                     uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_golay_encode_rows(const uint8_t *nibbles, int32_t *codewords, int64_t rows,
                                          int64_t d, int threads);
KVECC_API int kvecc_cpu_golay_decode_rows(const int32_t *codewords, uint8_t *nibbles, int64_t rows,
                                          int64_t d, uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_golay_encode_packed(const uint8_t *nibbles, uint8_t *codewords, int64_t m,
                                            int threads);
KVECC_API int kvecc_cpu_golay_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                            uint8_t *uncorrectable, int64_t m, uint64_t *stats,
                                            int threads);
KVECC_API int kvecc_cpu_hamming84_encode_packed(const uint8_t *nibbles, uint8_t *codewords,
                                                int64_t n, int threads);
KVECC_API int kvecc_cpu_hamming84_decode_packed(const uint8_t *codewords, uint8_t *nibbles,
                                                uint8_t *error_types, int64_t n, uint64_t *stats,
                                                int threads);
KVECC_API int kvecc_cpu_inject_u8(const uint8_t *in, uint8_t *out, uint8_t *counts, int64_t n,
                                  int n_bits, int64_t seed, float ber, int64_t global_n,
                                  int64_t offset0, uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_inject_i32(const int32_t *in, int32_t *out, uint8_t *counts, int64_t n,
                                   int n_bits, int64_t seed, float ber, int64_t global_n,
                                   int64_t offset0, uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_inject_u8_vectorized(const uint8_t *in, uint8_t *out, uint8_t *counts,
                                             int64_t n, int n_bits, int64_t seed, float ber,
                                             uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_inject_i32_vectorized(const int32_t *in, int32_t *out, uint8_t *counts,
                                              int64_t n, int n_bits, int64_t seed, float ber,
                                              uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_inject_rows_u8(const uint8_t *in, uint8_t *out, int64_t rows,
                                       int64_t row_len, int n_bits, int64_t seed_base, float ber,
                                       uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_inject_rows_i32(const int32_t *in, int32_t *out, int64_t rows,
                                        int64_t row_len, int n_bits, int64_t seed_base, float ber,
                                        uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_count_ne_u8(const uint8_t *a, const uint8_t *b, int64_t n, uint64_t *stats,
                                    int threads);
KVECC_API int kvecc_cpu_interpolate(const uint8_t *q, const uint8_t *err, uint8_t *out,
                                    int64_t outer, int64_t len, int64_t inner, int threads);
KVECC_API int kvecc_cpu_quantize_encode_rows(const void *x, int x_dtype, int codec,
                                             int scale_rule, uint8_t *cw, float *scales,
                                             int64_t rows, int64_t d, int threads);
KVECC_API int kvecc_cpu_decode_dequant_h84_rows(const uint8_t *cw, const float *scales, void *out,
                                                int out_dtype, int64_t rows, int64_t d,
                                                int zero_doubles, uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_shim_write(const void *k, const void *v, int x_dtype, int64_t batch,
                                   int64_t seq, int64_t hkv, int64_t d, int codec,
                                   int scale_rule, int n_bits,
                                   int inject, float ber, int64_t seed0, void *k_cache,
                                   void *v_cache, float *k_scales, float *v_scales,
                                   const int32_t *block_table, int64_t num_layers,
                                   int64_t block_size, int64_t layer, int threads);
KVECC_API int kvecc_cpu_shim_read(const void *k_cache, const void *v_cache, const float *k_scales,
                                  const float *v_scales, const int32_t *block_table, int64_t ctx,
                                  int64_t hkv, int64_t d, int64_t num_layers, int64_t block_size,
                                  int64_t layer, int codec, int interp, void *k_out, void *v_out,
                                  int out_dtype, uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_shim_read_batch(const void *k_cache, const void *v_cache,
                                        const float *k_scales, const float *v_scales,
                                        const int32_t *block_table, int64_t table_stride,
                                        int64_t batch, int64_t ctx, int64_t hkv, int64_t d,
                                        int64_t num_layers, int64_t block_size, int64_t layer,
                                        int codec, int interp, void *k_out, void *v_out,
                                        int out_dtype, uint64_t *stats, int threads);
KVECC_API int kvecc_cpu_paged_attention(const void *query, int q_dtype, const void *k_cache,
                                        const void *v_cache, const int32_t *block_table,
                                        const int32_t *context_lens, const float *k_scales,
                                        const float *v_scales, void *out, int64_t batch,
                                        int64_t heads, int64_t kv_heads, int64_t head_dim,
                                        int64_t num_blocks, int64_t num_layers, int64_t layer, int64_t block_size,
                                        int64_t max_blocks, int64_t max_context_len,
                                        float sm_scale, int codec, int threads);

#ifdef __cplusplus
}
#endif
#endif /* KVECC_H */
