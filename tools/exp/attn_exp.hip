// attn_exp.hip -- paged-attention experiments (NOT shipped): this file
// #includes csrc/attention.hip and launches its kernels in shapes the product
// does not: the matrix-core kernels for one query head per cache head (MHA,
// G = 1: one of the 16 MFMA columns used), with other split sizes.
// tools/exp/run_attn_exp.py times them against kvecc_paged_attention.
// kvecc_exp_paged_attention_packed: the packed-Golay MHA split kernel with VEC
// codewords per lane (the product: 4, 11 of 16 lanes busy at D = 128; 3: 15 of 16,
// 9-byte unaligned lane chunks realigned with v_alignbyte).
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/attention.hip"

namespace kvecc {
namespace exp {

template <int G>
static void launch_mfma_g(int codec, const AttnArgs &a, int64_t batch, hipStream_t st) {
  const dim3 grid((unsigned)a.nsplit, (unsigned)(batch * a.heads / G));
  if (codec == KVECC_CODEC_H84) {
    switch (a.d) {
      case 64: KVECC_LAUNCH((paged_attn_h84_mfma_kernel<64, G>), grid, dim3(kBlock), 0, st, a); break;
      default: KVECC_LAUNCH((paged_attn_h84_mfma_kernel<128, G>), grid, dim3(kBlock), 0, st, a); break;
    }
  } else if (codec == KVECC_CODEC_GOLAY_PACKED) {
    KVECC_LAUNCH((paged_attn_golay_mfma_kernel<G, true>), grid, dim3(kBlock), 0, st, a);
  } else {
    KVECC_LAUNCH((paged_attn_golay_mfma_kernel<G, false>), grid, dim3(kBlock), 0, st, a);
  }
  if (!a.ctr) launch_combine<__half>(a, batch, st);
}

}  // namespace exp
}  // namespace kvecc

// Golay MHA split kernel (fp16 queries, G = 1, fused combine) with the parity
// half as two 64-entry tables (sp = 1: 16.5 KiB of LDS instead of 32; sp = 3:
// no table gathers at all, a probe), u rows
// in flight (0: the product's), per_cu workgroups per CU in the split choice
template <int CODEC, int U, int DEC, int VEC0 = 0>
static void launch_gsp(const kvecc::AttnArgs &a, dim3 grid, hipStream_t st) {
  using namespace kvecc;
  constexpr int VEC = VEC0 ? VEC0 : CODEC == KVECC_CODEC_GOLAY ? kGolayVec : kGolayPackedVec;
  constexpr int W = VEC == 6 ? 8 : 16;  // lanes per token row: 43 codewords / VEC, rounded up to a power of two
  KVECC_LAUNCH((paged_attn_split_kernel<__half, CODEC, VEC, W, true, 1, U, DEC>), grid, dim3(kBlock), 0, st, a);
}


extern "C" {

// kvecc_paged_attention (fp16 queries, caches < 4 GiB) with the matrix-core
// kernels forced at G query heads per workgroup (G = 1 allowed) and `per_cu`
// workgroups per CU in the split choice; fused = 1: the fused combine
__attribute__((visibility("default"))) int kvecc_exp_paged_attention_mfma(
    int G, int per_cu, int fused, const void *query, const void *k_cache, const void *v_cache,
    const int32_t *block_table, const int32_t *context_lens, const float *k_scales, const float *v_scales, void *out,
    int64_t batch, int64_t heads, int64_t kv_heads, int64_t head_dim, int64_t num_blocks, int64_t num_layers,
    int64_t layer, int64_t block_size, int64_t max_blocks, int64_t max_context_len, float sm_scale, int codec,
    float *workspace, void *stream) {
  using namespace kvecc;
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
  const int64_t rows_total = num_blocks * num_layers * kv_heads * block_size;
  const int64_t cb = rows_total * (codec == KVECC_CODEC_H84 ? head_dim
                                   : codec == KVECC_CODEC_GOLAY_PACKED ? (int64_t)a.rowb
                                                                       : 4 * a.g);
  a.cache_bytes = (uint32_t)cb;
  a.scale_bytes = (uint32_t)(rows_total * 4);
  a.split = choose_split(batch * heads / G, max_context_len, per_cu);
  a.nsplit = cdiv(max_context_len, a.split);
  a.ctr = fused ? attn_counter_slot(stream) : nullptr;
  a.par = golay_parity_table_dev();
  a.cor = golay_correct_table_dev();
  a.atab = golay_attn_table_dev();
  a.atab_x = golay_attn_x_table_dev();
  hipStream_t st = as_stream(stream);
  switch (G) {
    case 1: exp::launch_mfma_g<1>(codec, a, batch, st); break;
    case 2: exp::launch_mfma_g<2>(codec, a, batch, st); break;
    default: exp::launch_mfma_g<4>(codec, a, batch, st); break;
  }
  return check_launch("exp_paged_attention_mfma");
}

// packed Golay, fp16 queries, G = 1, fused combine; vec 3 or 4 (32 / 33: 3 with 2 / 3 rows in flight)
__attribute__((visibility("default"))) int kvecc_exp_paged_attention_packed(
    int vec, int per_cu, const void *query, const void *k_cache, const void *v_cache, const int32_t *block_table,
    const int32_t *context_lens, const float *k_scales, const float *v_scales, void *out, int64_t batch,
    int64_t heads, int64_t kv_heads, int64_t head_dim, int64_t num_blocks, int64_t block_size, int64_t max_blocks,
    int64_t max_context_len, float sm_scale, float *workspace, void *stream) {
  using namespace kvecc;
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
  a.g = (head_dim + 2) / 3;
  a.rowb = (uint32_t)KVECC_GOLAY_PACKED_ROW(a.g);
  a.layers = 1;
  a.layer = 0;
  a.bs = block_size;
  a.max_blocks = max_blocks;
  a.sm_scale = sm_scale;
  a.empty_value = 0.0f;
  const int64_t rows_total = num_blocks * kv_heads * block_size;
  a.cache_bytes = (uint32_t)(rows_total * a.rowb);
  a.scale_bytes = (uint32_t)(rows_total * 4);
  a.split = choose_split(batch * heads, max_context_len, per_cu);
  a.nsplit = cdiv(max_context_len, a.split);
  a.ctr = attn_counter_slot(stream);
  a.par = golay_parity_table_dev();
  a.cor = golay_correct_table_dev();
  a.atab = golay_attn_table_dev();
  a.atab_x = golay_attn_x_table_dev();
  const dim3 grid((unsigned)a.nsplit, (unsigned)(batch * heads));
  hipStream_t st = as_stream(stream);
  if (vec == 3)
    KVECC_LAUNCH((paged_attn_split_kernel<__half, KVECC_CODEC_GOLAY_PACKED, 3, 16, true, 1>), grid, dim3(kBlock), 0,
                 st, a);
  else if (vec == 32)  // 3 codewords per lane, 2 rows in flight
    KVECC_LAUNCH((paged_attn_split_kernel<__half, KVECC_CODEC_GOLAY_PACKED, 3, 16, true, 1, 2>), grid, dim3(kBlock),
                 0, st, a);
  else if (vec == 33)  // 3 codewords per lane, 3 rows in flight
    KVECC_LAUNCH((paged_attn_split_kernel<__half, KVECC_CODEC_GOLAY_PACKED, 3, 16, true, 1, 3>), grid, dim3(kBlock),
                 0, st, a);
  else
    KVECC_LAUNCH((paged_attn_split_kernel<__half, KVECC_CODEC_GOLAY_PACKED, 4, 16, true, 1>), grid, dim3(kBlock), 0,
                 st, a);
  return check_launch("exp_paged_attention_packed");
}


__attribute__((visibility("default"))) int kvecc_exp_paged_attention_gsp(
    int packed, int sp, int u, int per_cu, const void *query, const void *k_cache, const void *v_cache,
    const int32_t *block_table, const int32_t *context_lens, const float *k_scales, const float *v_scales, void *out,
    int64_t batch, int64_t heads, int64_t kv_heads, int64_t head_dim, int64_t num_blocks, int64_t block_size,
    int64_t max_blocks, int64_t max_context_len, float sm_scale, float *workspace, void *stream) {
  using namespace kvecc;
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
  a.g = (head_dim + 2) / 3;
  a.rowb = (uint32_t)KVECC_GOLAY_PACKED_ROW(a.g);
  a.layers = 1;
  a.layer = 0;
  a.bs = block_size;
  a.max_blocks = max_blocks;
  a.sm_scale = sm_scale;
  a.empty_value = 0.0f;
  const int64_t rows_total = num_blocks * kv_heads * block_size;
  a.cache_bytes = (uint32_t)(rows_total * (packed ? (int64_t)a.rowb : 4 * a.g));
  a.scale_bytes = (uint32_t)(rows_total * 4);
  a.split = choose_split(batch * heads, max_context_len, per_cu);
  a.nsplit = cdiv(max_context_len, a.split);
  if (a.nsplit > kMaxSplits) return set_error(KVECC_EINVAL, "too many splits");
  a.ctr = attn_counter_slot(stream);
  a.par = golay_parity_table_dev();
  a.cor = golay_correct_table_dev();
  a.atab = golay_attn_table_dev();
  a.atab_x = golay_attn_x_table_dev();
  const dim3 grid((unsigned)a.nsplit, (unsigned)(batch * heads));
  hipStream_t st = as_stream(stream);
#define GSP(PK, UU, S)                                                                             \
  if (packed == PK && u == UU && sp == S) {                                                        \
    launch_gsp<PK ? KVECC_CODEC_GOLAY_PACKED : KVECC_CODEC_GOLAY, UU, (int)S>(a, grid, st);       \
    return check_launch("exp_paged_attention_gsp");                                                \
  }
  GSP(0, 0, false) GSP(0, 0, true) GSP(0, 3, true) GSP(0, 4, true) GSP(0, 3, false)
  // sp 2: 6 codewords per lane, 8 lanes per token row (int32), u rows in flight
  if (packed == 0 && sp == 2) {
    if (u == 1) launch_gsp<KVECC_CODEC_GOLAY, 1, false, 6>(a, grid, st);
    else if (u == 2) launch_gsp<KVECC_CODEC_GOLAY, 2, false, 6>(a, grid, st);
    else launch_gsp<KVECC_CODEC_GOLAY, 3, false, 6>(a, grid, st);
    return check_launch("exp_paged_attention_gsp");
  }
  GSP(1, 0, false) GSP(1, 0, true) GSP(1, 2, true) GSP(1, 3, true)
  // sp 3: the product's kernel with its decode's two LDS gathers skipped (WRONG values: prices them)
  if (sp == 3 && u == 0) {
    if (packed) launch_gsp<KVECC_CODEC_GOLAY_PACKED, 0, 2>(a, grid, st);
    else launch_gsp<KVECC_CODEC_GOLAY, 0, 2>(a, grid, st);
    return check_launch("exp_paged_attention_gsp");
  }
#undef GSP
  return set_error(KVECC_EINVAL, "no gsp instance");
}

}  // extern "C"
