// h84_pk_enc_exp.hip -- experimental grids for the packed Hamming(8,4) encode
// (csrc/packed.hip h84_encode_packed_kernel), NOT shipped.  #includes packed.hip;
// tools/exp/run_h84_pk_enc_exp.py times the variants against
// kvecc_hamming84_encode_packed in one process and compares the bytes.
//   v 0: the product's grid-stride loop at per_cu workgroups per CU
//   v 1: a full grid, one 16-value chunk per lane (no stride loop)
//   v 2: a full grid, two chunks per lane (one 16-byte nibble load, two 16-byte stores)
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/packed.hip"

namespace kvecc {
namespace exp {

__global__ __launch_bounds__(kHpBlock) void h84_pk_enc_full_kernel(const u32x2 *__restrict__ nib, u32x4 *__restrict__ cw,
                                                                   int64_t n16) {
  const int64_t i = (int64_t)blockIdx.x * kHpBlock + threadIdx.x;
  if (i >= n16) return;
  const u32x2 v = ld_stream(nib + i);
  st_stream(cw + i, u32x4{h84_encode4(nib_unpack4(v.x & 0xFFFFu)), h84_encode4(nib_unpack4(v.x >> 16)),
                          h84_encode4(nib_unpack4(v.y & 0xFFFFu)), h84_encode4(nib_unpack4(v.y >> 16))});
}

// lane l of a wave covers chunks base + l and base + 64 + l (each wave-instruction
// stays 1 KiB contiguous on the store side)
__global__ __launch_bounds__(kHpBlock) void h84_pk_enc_full2_kernel(const u32x2 *__restrict__ nib,
                                                                    u32x4 *__restrict__ cw, int64_t n16) {
  const int64_t w = ((int64_t)blockIdx.x * kHpBlock + threadIdx.x) / kWave;
  const int64_t lane = threadIdx.x % kWave;
  const int64_t i0 = w * 2 * kWave + lane, i1 = i0 + kWave;
  u32x2 a = {0u, 0u}, b = {0u, 0u};
  if (i0 < n16) a = ld_stream(nib + i0);
  if (i1 < n16) b = ld_stream(nib + i1);
  if (i0 < n16)
    st_stream(cw + i0, u32x4{h84_encode4(nib_unpack4(a.x & 0xFFFFu)), h84_encode4(nib_unpack4(a.x >> 16)),
                             h84_encode4(nib_unpack4(a.y & 0xFFFFu)), h84_encode4(nib_unpack4(a.y >> 16))});
  if (i1 < n16)
    st_stream(cw + i1, u32x4{h84_encode4(nib_unpack4(b.x & 0xFFFFu)), h84_encode4(nib_unpack4(b.x >> 16)),
                             h84_encode4(nib_unpack4(b.y & 0xFFFFu)), h84_encode4(nib_unpack4(b.y >> 16))});
}

// C chunks per lane, lane l of a wave at base + 64 c + l: all C loads first
template <int C>
__global__ __launch_bounds__(kHpBlock) void h84_pk_enc_fullc_kernel(const u32x2 *__restrict__ nib,
                                                                    u32x4 *__restrict__ cw, int64_t n16) {
  const int64_t w = ((int64_t)blockIdx.x * kHpBlock + threadIdx.x) / kWave;
  const int64_t lane = threadIdx.x % kWave;
  const int64_t i0 = w * C * kWave + lane;
  u32x2 a[C];
#pragma unroll
  for (int c = 0; c < C; ++c) a[c] = i0 + kWave * c < n16 ? ld_stream(nib + i0 + kWave * c) : u32x2{0u, 0u};
#pragma unroll
  for (int c = 0; c < C; ++c)
    if (i0 + kWave * c < n16)
      st_stream(cw + i0 + kWave * c,
                u32x4{h84_encode4(nib_unpack4(a[c].x & 0xFFFFu)), h84_encode4(nib_unpack4(a[c].x >> 16)),
                      h84_encode4(nib_unpack4(a[c].y & 0xFFFFu)), h84_encode4(nib_unpack4(a[c].y >> 16))});
}

}  // namespace exp
}  // namespace kvecc

extern "C" __attribute__((visibility("default"))) int kvecc_exp_h84_pk_enc(int v, int per_cu, const uint8_t *nibbles,
                                                                          uint8_t *codewords, int64_t n, void *stream) {
  using namespace kvecc;
  if (n % 16 || !aligned(nibbles, 8) || !aligned(codewords, 16)) return set_error(KVECC_EINVAL, "exp: n %% 16, alignment");
  const int64_t n16 = n / 16;
  hipStream_t st = as_stream(stream);
  auto in = reinterpret_cast<const u32x2 *>(nibbles);
  auto out = reinterpret_cast<u32x4 *>(codewords);
  if (v == 0)
    KVECC_LAUNCH(h84_encode_packed_kernel, dim3(grid_for(n16, kHpBlock, per_cu)), dim3(kHpBlock), 0, st, in, out, n16);
  else if (v == 1)
    KVECC_LAUNCH(exp::h84_pk_enc_full_kernel, dim3((unsigned)cdiv(n16, kHpBlock)), dim3(kHpBlock), 0, st, in, out, n16);
  else if (v == 3)
    KVECC_LAUNCH(exp::h84_pk_enc_fullc_kernel<4>, dim3((unsigned)cdiv(n16, 4 * kHpBlock)), dim3(kHpBlock), 0, st, in,
                 out, n16);
  else if (v == 4)
    KVECC_LAUNCH(exp::h84_pk_enc_fullc_kernel<2>, dim3((unsigned)cdiv(n16, 2 * kHpBlock)), dim3(kHpBlock), 0, st, in,
                 out, n16);
  else
    KVECC_LAUNCH(exp::h84_pk_enc_full2_kernel, dim3((unsigned)cdiv(n16, 2 * kHpBlock)), dim3(kHpBlock), 0, st, in, out,
                 n16);
  return check_launch("exp_h84_pk_enc");
}

// the packed Golay encode (golay_encode_packed_kernel) at per_cu workgroups per
// CU (the product: 16); m a multiple of its tile
extern "C" __attribute__((visibility("default"))) int kvecc_exp_gpk_enc(int per_cu, const uint8_t *nibbles,
                                                                       uint8_t *codewords, int64_t m, void *stream) {
  using namespace kvecc;
  if (m % kPkTile) return set_error(KVECC_EINVAL, "exp: m %% tile");
  const uint16_t *par = golay_parity_table_dev();
  if (!par) return KVECC_EHIP;
  const int64_t ntiles = m / kPkTile;
  KVECC_LAUNCH(golay_encode_packed_kernel, dim3(grid_for(ntiles, 1, per_cu)), dim3(kPkBlock), 0, as_stream(stream),
               reinterpret_cast<const uint32_t *>(nibbles), reinterpret_cast<uint32_t *>(codewords), ntiles, par);
  return check_launch("exp_gpk_enc");
}
