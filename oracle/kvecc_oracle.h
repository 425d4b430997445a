/*
 * kvecc_oracle.h -- CPU restatement of the reference ECC codec path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline).  The product (libkvecc.so) never links it.
 *
 * Parity status: PINNED.  Every function here is checked by tests/test_oracle.py
 * against golden vectors in tests/golden/ that tools/gen_golden.py produced by
 * running the reference's own @triton.jit kernels under TRITON_INTERPRET=1.
 *
 * Every function cites the reference file:line it restates
 * (paths relative to the reference repository root).
 */
#ifndef KVECC_ORACLE_H
#define KVECC_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ecc_codecs/triton_kernels/config.py:354-379 (_compute_golay_h_row_masks) */
void oracle_golay_h_row_masks(uint32_t out[12]);
/* ecc_codecs/triton_kernels/config.py:403-457 (build_golay_syndrome_table) */
void oracle_golay_syndrome_table(int32_t out[4096]);

/* hamming74_triton.py:48-91 */
void oracle_h74_encode(const uint8_t *in, uint8_t *out, int64_t n);
/* hamming74_triton.py:100-162 + wrapper stats :269 ; stats[0] = #syndrome!=0 */
void oracle_h74_decode(const uint8_t *cw, uint8_t *data, uint8_t *flag, int64_t n,
                       int64_t *stats);
/* hamming84_triton.py:50-108 */
void oracle_h84_encode(const uint8_t *in, uint8_t *out, int64_t n);
/* hamming84_triton.py:117-209 + wrapper stats :341-342 ; stats = {#type1, #type2} */
void oracle_h84_decode(const uint8_t *cw, uint8_t *data, uint8_t *etype, int64_t n,
                       int64_t *stats);

/* golay_triton.py:99-157 ; triplets uint8[m*3] -> int32[m] */
void oracle_golay_encode(const uint8_t *trip, int32_t *cw, int64_t m);
/* golay_triton.py:213-295 + wrapper stats :491-493 ; stats = {sum count<4, #count==4} */
void oracle_golay_decode(const int32_t *cw, uint8_t *trip, uint8_t *count, int64_t m,
                         int64_t *stats);

/* triton/language/random.py:12-110 : Philox4x32-10, returns the 4 output words */
void oracle_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                          uint32_t k0, uint32_t k1, uint32_t out[4]);
/* triton/language/random.py:126-143 : uint32 -> float32 in [0,1) */
float oracle_uint_to_uniform(uint32_t x);

/*
 * fault_injection_triton.py:228-299 (uint8) / :303-334 (int32), launched by
 * inject_bit_errors_triton :337-424.  Element i of this call is global element
 * (offset0 + i) of a tensor of global_n elements, so a shard reproduces the
 * unsharded flip pattern.  stats = {total flips, elements with >=1 flip}.
 */
void oracle_inject_u8(const uint8_t *in, uint8_t *out, uint8_t *count, int64_t n,
                      int n_bits, int64_t seed, float ber, int64_t global_n,
                      int64_t offset0, int64_t *stats);
void oracle_inject_rows_u8(const uint8_t *in, uint8_t *out, int64_t rows, int64_t row_len,
                           int n_bits, int64_t seed0, float ber, int64_t *stats);
void oracle_inject_i32(const int32_t *in, int32_t *out, uint8_t *count, int64_t n,
                       int n_bits, int64_t seed, float ber, int64_t global_n,
                       int64_t offset0, int64_t *stats);
/* fault_injection_triton.py:57-133 / :137-224 (rand4x variants) */
void oracle_inject_u8_vectorized(const uint8_t *in, uint8_t *out, uint8_t *count,
                                 int64_t n, int n_bits, int64_t seed, float ber,
                                 int64_t *stats);
void oracle_inject_i32_vectorized(const int32_t *in, int32_t *out, uint8_t *count,
                                  int64_t n, int n_bits, int64_t seed, float ber,
                                  int64_t *stats);

/*
 * interpolation_triton.py:120-159 kernel semantics on an [outer, len, inner]
 * contiguous array, the sequence axis being the middle one (every element is
 * clamped to [0,15]; the wrapper's no-double fast path is the caller's job).
 */
void oracle_interpolate(const uint8_t *q, const uint8_t *err, uint8_t *out,
                        int64_t outer, int64_t len, int64_t inner);

/*
 * Shim quantization (kv_cache/ecc_shim.py:572-580 with
 * kv_cache/paged_cache_ecc.py:302-334): per row of d fp32 values,
 * scale = absmax/7 (0 -> 1), q = round_half_even(x/scale) clamped [-8,7] + 8.
 * rule 0: the scale by IEEE division (torch on CPU tensors, the golden
 * fixtures); rule 1: absmax * RN(1/7) (torch's tensor / Python scalar on a GPU).
 */
void oracle_quantize_rows(const float *x, int64_t rows, int64_t d, int rule, uint8_t *q,
                          float *scales);
/* fused_kernels.py:272-357 data path: H84 decode, doubles -> 0, (q-8)*scale */
void oracle_decode_dequant_h84(const uint8_t *cw, const float *scales, int64_t rows,
                               int64_t d, float *out, int64_t *corrected);

#ifdef __cplusplus
}
#endif
#endif
