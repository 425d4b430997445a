// golay_exp3.hip -- decode refinements on the G=2/BS=512 winner:
//   P: parity via LDS table (0) or VALU (1, 12 x bitfield-extract + 3-input xor-and)
//   S: direct dwordx3+dword stores (0) or LDS-staged dwordx4 stores (1)
#include "../../quantized-kv-cache-ecc-protection_amd/csrc/kvecc_internal.h"

using namespace kvecc;

__device__ __forceinline__ uint32_t spread_nibbles(uint32_t d) {
  return (d & 0xFu) | (d & 0xF0u) << 4 | (d & 0xF00u) << 8;
}

__device__ __forceinline__ uint32_t parity_valu(uint32_t d) {
  constexpr uint32_t R[12] = {0xA3B, 0xD1D, 0xE8E, 0xB47, 0xDA3, 0xED1,
                              0xF68, 0xBB4, 0x9DA, 0x8ED, 0xC76, 0x7FF};
  uint32_t p = 0;
#pragma unroll
  for (int j = 0; j < 12; ++j) p ^= (uint32_t)(-(int32_t)((d >> j) & 1u)) & R[j];
  return p;
}

template <int BS, int P, int S>
__global__ __launch_bounds__(BS) void dec3(const u32x4 *__restrict__ cw, uint8_t *__restrict__ trip8,
                                           uint8_t *__restrict__ counts8, int64_t ntiles,
                                           const uint16_t *__restrict__ par, const uint16_t *__restrict__ cor,
                                           uint64_t *__restrict__ stats) {
  constexpr int G = 2;
  constexpr int WCW = 64 * G * 4;  // codewords per wave per tile (512)
  __shared__ __attribute__((aligned(16))) uint16_t cor_lds[4096];
  __shared__ __attribute__((aligned(16))) uint16_t par_lds[P == 0 ? 4096 : 8];
  __shared__ __attribute__((aligned(16))) uint32_t stage[S ? (BS / 64) * (WCW * 4 / 4) : 4];
  {
    const u32x4 *c = reinterpret_cast<const u32x4 *>(cor);
    const u32x4 *p = reinterpret_cast<const u32x4 *>(par);
    for (int i = threadIdx.x; i < 512; i += BS) {
      reinterpret_cast<u32x4 *>(cor_lds)[i] = c[i];
      if (P == 0) reinterpret_cast<u32x4 *>(par_lds)[i] = p[i];
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t *stw = stage + (S ? wave * WCW : 0);  // per-wave region: 3*WCW/4 trip words + WCW/4 count words
  uint32_t bits = 0, unc = 0;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int64_t wbase = t * (BS / 64) * WCW + wave * WCW;  // first codeword of this wave
    const int64_t base = wbase + lane * 4;
    u32x4 v[G];
#pragma unroll
    for (int g = 0; g < G; ++g) v[g] = __builtin_nontemporal_load(cw + (base + g * 256) / 4);
#pragma unroll
    for (int g = 0; g < G; ++g) {
      uint32_t c[4], e[4];
      const uint32_t w[4] = {v[g].x, v[g].y, v[g].z, v[g].w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t lo = w[k] & 0xFFFu;
        uint32_t p = P == 0 ? (uint32_t)par_lds[lo] : parity_valu(lo);
        uint32_t ee = cor_lds[((w[k] >> 12) & 0xFFFu) ^ p];
        c[k] = ee >> 12;
        e[k] = spread_nibbles(lo ^ (ee & 0xFFFu));
      }
      const uint32_t t0 = e[0] | e[1] << 24, t1 = e[1] >> 8 | e[2] << 16, t2 = e[2] >> 16 | e[3] << 8;
      const uint32_t cc = c[0] | c[1] << 8 | c[2] << 16 | c[3] << 24;
      if (S) {
        // wave-local byte offsets: triplets at 3*(g*256 + 4*lane), counts after 3*WCW
        const int tw = (3 * (g * 256 + 4 * lane)) / 4;
        stw[tw] = t0;
        stw[tw + 1] = t1;
        stw[tw + 2] = t2;
        stw[3 * WCW / 4 + (g * 256 + 4 * lane) / 4] = cc;
      } else {
        uint32_t *p = reinterpret_cast<uint32_t *>(trip8 + (base + g * 256) * 3);
        __builtin_nontemporal_store(t0, p);
        __builtin_nontemporal_store(t1, p + 1);
        __builtin_nontemporal_store(t2, p + 2);
        __builtin_nontemporal_store(cc, reinterpret_cast<uint32_t *>(counts8 + base + g * 256));
      }
      bits += ((cc & 0x03030303u) * 0x01010101u) >> 24;
      unc += __builtin_popcount(cc & 0x04040404u);
    }
    if (S) {
      // wave region = 4*WCW bytes = 2048 B = 2 instructions of 64 lanes x 16 B:
      // instruction 0 -> triplet bytes [0,1024), instruction 1 -> lanes 0..31 triplet
      // bytes [1024,1536), lanes 32..63 count bytes [0,512)
      __builtin_amdgcn_wave_barrier();
      const u32x4 *sv = reinterpret_cast<const u32x4 *>(stw);
      u32x4 a = sv[lane], b = sv[64 + lane];
      __builtin_nontemporal_store(a, reinterpret_cast<u32x4 *>(trip8 + wbase * 3) + lane);
      if (lane < 32)
        __builtin_nontemporal_store(b, reinterpret_cast<u32x4 *>(trip8 + wbase * 3) + 64 + lane);
      else
        __builtin_nontemporal_store(b, reinterpret_cast<u32x4 *>(counts8 + wbase) + (lane - 32));
      __builtin_amdgcn_wave_barrier();
    }
  }
  __shared__ uint32_t red[2][BS / 64];
  for (int off = 32; off > 0; off >>= 1) {
    bits += __shfl_xor(bits, off, 64);
    unc += __shfl_xor(unc, off, 64);
  }
  if (lane == 0) { red[0][wave] = bits; red[1][wave] = unc; }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long a = 0, b = 0;
    for (int i = 0; i < BS / 64; ++i) { a += red[0][i]; b += red[1][i]; }
    uint64_t *slot = stats + (blockIdx.x % 32) * 16;
    if (a) atomicAdd(reinterpret_cast<unsigned long long *>(slot), a);
    if (b) atomicAdd(reinterpret_cast<unsigned long long *>(slot + 1), b);
  }
}

#define D3(BS, P, S) hipLaunchKernelGGL((dec3<BS, P, S>), dim3(grid), dim3(BS), 0, st, C, T, N, m / ((BS / 64) * 512), par, cor, stats)

extern "C" __attribute__((visibility("default"))) int exp3_decode(int variant, const int32_t *cw, uint8_t *T,
                                                                  uint8_t *N, int64_t m, uint64_t *stats,
                                                                  const uint16_t *tables, int grid, void *stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const uint16_t *par = tables, *cor = tables + 4096;
  auto C = reinterpret_cast<const u32x4 *>(cw);
  switch (variant) {
    case 0: D3(512, 0, 0); break;
    case 1: D3(512, 1, 0); break;
    case 2: D3(512, 0, 1); break;
    case 3: D3(512, 1, 1); break;
    case 4: D3(1024, 0, 0); break;
    case 5: D3(1024, 1, 0); break;
    case 6: D3(1024, 1, 1); break;
    case 7: D3(256, 1, 0); break;
    case 8: D3(256, 1, 1); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
