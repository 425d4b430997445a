// runtime.hip -- error reporting, device queries and the Golay code tables.
//
// The Golay tables are built here on the host, from the code's definition
// (the B matrix of ecc_codecs/triton_kernels/config.py:329-347), and uploaded
// once per device; they replace the per-device syndrome-table cache of
// golay_triton.py:304-330.
#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <mutex>

#include "kvecc_internal.h"

namespace kvecc {

static thread_local char g_err[512] = "";
thread_local LaunchTiming g_launch_timing = {nullptr, nullptr};

int set_error(int code, const char *fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}

int check_launch(const char *what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error(KVECC_EHIP, "%s: %s", what, hipGetErrorString(e));
  return KVECC_OK;
}

constexpr int kMaxDev = 64;
static std::mutex g_mu;
static int g_cu[kMaxDev];
static std::atomic<uint16_t *> g_parity[kMaxDev];
static std::atomic<uint16_t *> g_correct[kMaxDev];
static std::atomic<uint32_t *> g_attn[kMaxDev];
static std::atomic<uint8_t *> g_pk[kMaxDev];
static std::atomic<uint32_t *> g_dyn[kMaxDev];  // kDynSlots work-counter slots, zeroed
static std::atomic<uint32_t> g_dyn_next[kMaxDev];
static std::atomic<uint32_t *> g_actr[kMaxDev];  // kAttnCtrSlots attention split counters, zeroed
static std::atomic<uint32_t> g_actr_next[kMaxDev];

int current_device() {
  int d = 0;
  if (hipGetDevice(&d) != hipSuccess) return 0;
  return d;
}

int cu_count() {
  int d = current_device();
  if (d < 0 || d >= kMaxDev) return 256;
  int c = __atomic_load_n(&g_cu[d], __ATOMIC_ACQUIRE);
  if (c > 0) return c;
  int v = 0;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || v <= 0)
    v = 256;
  __atomic_store_n(&g_cu[d], v, __ATOMIC_RELEASE);
  return v;
}

// Rows of B as 12-bit masks (bit i of row j = B[j][i]); B is symmetric, so
// these are also its columns, the reference's B_COL_* (golay_triton.py:59-70).
static const uint16_t kGolayRow[12] = {0xA3B, 0xD1D, 0xE8E, 0xB47, 0xDA3, 0xED1,
                                       0xF68, 0xBB4, 0x9DA, 0x8ED, 0xC76, 0x7FF};

void build_golay_parity_table(uint16_t *out) {
  // parity(d) = XOR of the B rows of the set data bits (linear code)
  for (uint32_t d = 0; d < 4096; ++d) {
    uint32_t p = 0;
    for (int j = 0; j < 12; ++j)
      if (d >> j & 1u) p ^= kGolayRow[j];
    out[d] = (uint16_t)p;
  }
}

static inline uint32_t syndrome24(uint32_t w, const uint16_t *par) {
  // H = [B^T | I]  =>  syndrome = parity bits received ^ parity(data received)
  return ((w >> 12) & 0xFFFu) ^ par[w & 0xFFFu];
}

// error pattern per syndrome exactly as config.py:403-457 orders it
static void build_error_patterns(int32_t *pat) {
  uint16_t par[4096];
  build_golay_parity_table(par);
  for (int s = 0; s < 4096; ++s) pat[s] = -1;
  pat[0] = 0;
  for (int i = 0; i < 24; ++i) pat[syndrome24(1u << i, par)] = (int32_t)(1u << i);
  for (int i = 0; i < 24; ++i)
    for (int j = i + 1; j < 24; ++j) {
      uint32_t e = (1u << i) | (1u << j);
      uint32_t s = syndrome24(e, par);
      if (pat[s] < 0) pat[s] = (int32_t)e;
    }
  for (int i = 0; i < 24; ++i)
    for (int j = i + 1; j < 24; ++j)
      for (int k = j + 1; k < 24; ++k) {
        uint32_t e = (1u << i) | (1u << j) | (1u << k);
        uint32_t s = syndrome24(e, par);
        if (pat[s] < 0) pat[s] = (int32_t)e;
      }
}

void build_golay_correct_table(uint16_t *out) {
  int32_t pat[4096];
  build_error_patterns(pat);
  for (int s = 0; s < 4096; ++s) {
    if (pat[s] < 0) {
      out[s] = (uint16_t)(4u << 12);  // uncorrectable: data kept, count 4
    } else {
      uint32_t e = (uint32_t)pat[s];
      out[s] = (uint16_t)((e & 0xFFFu) | ((uint32_t)__builtin_popcount(e) << 12));
    }
  }
}

static uint32_t spread12(uint32_t x) { return (x & 0xFu) | (x >> 4 & 0xFu) << 8 | (x >> 8 & 0xFu) << 16; }

// All Golay device tables of a device in one allocation, built together the
// first time any of them is needed (kvecc_init_device builds them eagerly, so
// no upload ever happens inside a HIP-graph capture): parity[4096] and
// correct[4096] as uint16, then the attention spread tables (uint32[8192]).
// The pointers are published through atomics after the upload completes.
static int ensure_tables(int d) {
  if (d < 0 || d >= kMaxDev) return set_error(KVECC_EINVAL, "device %d out of range", d);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_attn[d].load(std::memory_order_acquire)) return KVECC_OK;
  struct Host {
    uint16_t par[4096], cor[4096];
    uint32_t attn[8192];
    uint16_t pk0[4096];  // packed decode: parity(lo) << 2 (byte offset of the syndrome's entry)
    uint32_t pk1[4096];  // packed decode: error data | (bits & 3) << 24 | uncorrectable << 31
  };
  static_assert(offsetof(Host, pk1) == offsetof(Host, pk0) + 8192, "packed tables contiguous");
  static Host host;  // guarded by g_mu
  build_golay_parity_table(host.par);
  build_golay_correct_table(host.cor);
  for (uint32_t i = 0; i < 4096; ++i) {
    host.attn[i] = spread12(i) | (uint32_t)host.par[i] << 20;
    // correction half: data bits of the error pattern spread one nibble per
    // byte; byte 3 = (bits corrected & 3) | uncorrectable << 6 (count 4 -> 0x40),
    // so a sum of byte 3 over up to 21 codewords keeps both fields apart
    const uint32_t n = host.cor[i] >> 12;  // 0-3 bits corrected, 4 = uncorrectable
    host.attn[4096 + i] = spread12(host.cor[i] & 0xFFFu) | ((n & 3u) | (n >> 2) << 6) << 24;
    host.pk0[i] = (uint16_t)(host.par[i] << 2);
    host.pk1[i] = (host.cor[i] & 0xFFFu) | (n & 3u) << 24 | (n >> 2) << 31;
  }
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return set_error(KVECC_ENODEV, "hipGetDevice failed");
  if (hipSetDevice(d) != hipSuccess) return set_error(KVECC_ENODEV, "hipSetDevice(%d) failed", d);
  Host *buf = nullptr;
  uint32_t *dyn = nullptr;
  const size_t dyn_bytes = sizeof(uint32_t) * kDynSlots * kDynSlotWords;
  hipError_t e = hipMalloc(&buf, sizeof(Host));
  if (e == hipSuccess) e = hipMemcpy(buf, &host, sizeof(Host), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&dyn, dyn_bytes);
  if (e == hipSuccess) e = hipMemset(dyn, 0, dyn_bytes);
  uint32_t *actr = nullptr;
  const size_t actr_bytes = sizeof(uint32_t) * kAttnCtrSlots * kAttnCtrPerSlot;
  if (e == hipSuccess) e = hipMalloc(&actr, actr_bytes);
  if (e == hipSuccess) e = hipMemset(actr, 0, actr_bytes);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return set_error(KVECC_EHIP, "golay table upload: %s", hipGetErrorString(e));
  g_dyn[d].store(dyn, std::memory_order_release);
  g_actr[d].store(actr, std::memory_order_release);
  g_parity[d].store(buf->par, std::memory_order_release);
  g_correct[d].store(buf->cor, std::memory_order_release);
  g_pk[d].store(reinterpret_cast<uint8_t *>(buf->pk0), std::memory_order_release);
  g_attn[d].store(buf->attn, std::memory_order_release);  // last: the "built" flag
  return KVECC_OK;
}

template <typename P>
static const P *table_dev(std::atomic<P *> *tabs) {
  const int d = current_device();
  if (d >= 0 && d < kMaxDev && g_attn[d].load(std::memory_order_acquire)) return tabs[d].load(std::memory_order_acquire);
  if (ensure_tables(d) != KVECC_OK) return nullptr;
  return tabs[d].load(std::memory_order_acquire);
}

const uint16_t *golay_parity_table_dev() { return table_dev(g_parity); }
const uint16_t *golay_correct_table_dev() { return table_dev(g_correct); }
const uint32_t *golay_attn_table_dev() { return table_dev(g_attn); }
const uint8_t *golay_pk_table_dev() { return table_dev(g_pk); }

uint32_t *shim_dyn_slot() {
  const int d = current_device();
  if (!table_dev(g_attn)) return nullptr;  // allocated with the tables
  const uint32_t k = g_dyn_next[d].fetch_add(1, std::memory_order_relaxed) % kDynSlots;
  return g_dyn[d].load(std::memory_order_acquire) + (size_t)k * kDynSlotWords;
}

uint32_t *attn_counter_slot() {
  const int d = current_device();
  if (!table_dev(g_attn)) return nullptr;  // allocated with the tables
  const uint32_t k = g_actr_next[d].fetch_add(1, std::memory_order_relaxed) % kAttnCtrSlots;
  return g_actr[d].load(std::memory_order_acquire) + (size_t)k * kAttnCtrPerSlot;
}

}  // namespace kvecc

using namespace kvecc;

extern "C" {

KVECC_API const char *kvecc_version(void) { return "kvecc 0.1.0 (gfx950)"; }

KVECC_API const char *kvecc_last_error(void) { return g_err; }

KVECC_API int kvecc_time_next_launch(void *start_event, void *stop_event) {
  g_launch_timing = {reinterpret_cast<hipEvent_t>(start_event),
                     reinterpret_cast<hipEvent_t>(stop_event)};
  return KVECC_OK;
}

KVECC_API int kvecc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

KVECC_API int kvecc_init_device(int device) {
  int n = kvecc_device_count();
  if (n <= 0) return set_error(KVECC_ENODEV, "no HIP device visible");
  if (device < 0 || device >= n) return set_error(KVECC_EINVAL, "device %d not in [0,%d)", device, n);
  return ensure_tables(device);
}

KVECC_API int kvecc_golay_syndrome_table_host(int32_t *out) {
  if (!out) return set_error(KVECC_EINVAL, "null output");
  build_error_patterns(out);
  return KVECC_OK;
}

KVECC_API int kvecc_golay_h_row_masks_host(uint32_t *out) {
  if (!out) return set_error(KVECC_EINVAL, "null output");
  for (int i = 0; i < 12; ++i) out[i] = (uint32_t)kGolayRow[i] | (1u << (12 + i));
  return KVECC_OK;
}

KVECC_API uint32_t kvecc_ber_threshold(float ber) {
  // flip(x) := fp32(x) * 4.6566127342e-10f < ber is a prefix of [0, 2^31):
  // both the int->float conversion and the multiply round monotonically.
  const float scale = 4.6566127342e-10f;
  uint32_t lo = 0, hi = 0x80000000u;  // answer in [lo, hi]
  while (lo < hi) {
    uint32_t mid = lo + (hi - lo) / 2;
    volatile float u = (float)(int32_t)mid * scale;
    if (u < ber)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

}  // extern "C"
