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
#include <functional>
#include <map>
#include <mutex>
#include <thread>
#include <unordered_map>
#include <vector>

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
static std::atomic<uint32_t *> g_attn_x[kMaxDev];
static std::atomic<uint8_t *> g_pk[kMaxDev];

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
static uint32_t spread12x(uint32_t x) { return (x & 0xFu) | (x >> 4 & 0xFu) << 8 | (x >> 8 & 0xFu) << 28; }

// All Golay device tables of a device in one allocation, built together the
// first time any of them is needed (kvecc_init_device builds them eagerly, so
// no upload ever happens inside a HIP-graph capture): parity[4096] and
// correct[4096] as uint16, then the attention spread tables (uint32[8192], two
// layouts).
// The pointers are published through atomics after the upload completes.
static int ensure_tables(int d) {
  if (d < 0 || d >= kMaxDev) return set_error(KVECC_EINVAL, "device %d out of range", d);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_attn[d].load(std::memory_order_acquire)) return KVECC_OK;
  struct Host {
    uint16_t par[4096], cor[4096];
    uint32_t attn[8192];
    uint32_t attn_x[8192];  // attention-only variant: parity at the codeword's parity bits
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
    // the attention split kernels' variant, for words holding codeword << 2:
    // data nibbles at bits 0-3, 8-11 and 28-31, parity(lo) at bits 14-25 --
    // where such a word holds the received parity -- so the syndrome's byte
    // offset is one masked XOR and a shift
    host.attn_x[i] = spread12x(i) | (uint32_t)host.par[i] << 14;
    host.attn_x[4096 + i] = spread12x(host.cor[i] & 0xFFFu);
    host.pk0[i] = (uint16_t)(host.par[i] << 2);
    host.pk1[i] = (host.cor[i] & 0xFFFu) | (n & 3u) << 24 | (n >> 2) << 31;
  }
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return set_error(KVECC_ENODEV, "hipGetDevice failed");
  if (hipSetDevice(d) != hipSuccess) return set_error(KVECC_ENODEV, "hipSetDevice(%d) failed", d);
  Host *buf = nullptr;
  hipError_t e = hipMalloc(&buf, sizeof(Host));
  if (e == hipSuccess) e = hipMemcpy(buf, &host, sizeof(Host), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return set_error(KVECC_EHIP, "golay table upload: %s", hipGetErrorString(e));
  g_parity[d].store(buf->par, std::memory_order_release);
  g_correct[d].store(buf->cor, std::memory_order_release);
  g_pk[d].store(reinterpret_cast<uint8_t *>(buf->pk0), std::memory_order_release);
  g_attn_x[d].store(buf->attn_x, std::memory_order_release);
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
const uint32_t *golay_attn_x_table_dev() { return table_dev(g_attn_x); }
const uint8_t *golay_pk_table_dev() { return table_dev(g_pk); }

// ---- counter slots of the dynamically scheduled kernels -------------------------
// A kernel that takes work from counters (TileSchedule) or counts finished
// splits (the paged-attention fused combine) needs its counters zero at launch
// and to itself until it exits; it leaves them zero (each counter's last user
// resets it).  Both hold by stream order if a slot is never shared between
// launches that can overlap:
//   - eager launches: one slot per stream (per thread for hipStreamPerThread),
//     so consecutive users of a slot are ordered by their stream.  A slot is
//     keyed by the stream's address: a new stream created at a destroyed
//     stream's address inherits its slot, which is safe because
//     hipStreamDestroy drains the stream's queue before it returns (the old
//     stream's launches are done).  (hipStreamGetId would tell the two apart,
//     but it is a HIP 7.1 symbol and torch's HIP runtime here is 7.0);
//   - launches captured into a graph: a slot of their own per (capture, stream).
//     The slot is tied to the graph by a HIP user object: when the graph and
//     every executable instance of it are gone (and their launches done) the
//     runtime drops the last reference and the slot returns to the pool, zero
//     (every launch left it so).  Replays never share with eager work or other
//     graphs (replaying ONE graph concurrently with itself would race on its
//     outputs anyway).
// Slots come zeroed from a pool that grows outside captures only: every eager
// call tops the free list back up to kSlotReserve slots, so up to that many
// graphs can be captured between two eager launches (kvecc_reserve_counter_slots
// for more).  Growth zeroes a new chunk on a private stream (no device-wide sync).
struct SlotPool {
  std::mutex mu;
  std::vector<uint32_t *> free;                        // zeroed, never handed out
  std::unordered_map<uint64_t, uint32_t *> eager;      // stream key -> slot
  std::map<std::pair<uint64_t, unsigned long long>, uint32_t *> captured;  // (stream, capture id) -> slot
  std::vector<uint32_t *> chunks;
  hipStream_t side = nullptr;                          // zeroes new chunks
  // slots released by graph user objects: the runtime's destructor callback
  // only appends here (its own lock, no HIP call under it); counter_slot moves
  // them back to `free` under `mu`
  std::mutex ret_mu;
  std::vector<uint32_t *> returned;
};
// never destroyed: a graph user object's destructor (release_captured_slot)
// may run from a HIP runtime thread or during runtime teardown at exit, after
// static destructors; a heap array outlives both
static SlotPool *const g_pool = new SlotPool[kMaxDev];
// test hook (kvecc_debug_fail_graph_retain): make the graph-retain step of a
// capture's slot fail, to exercise that branch
static std::atomic<int> g_fail_retain{0};
constexpr int kSlotChunk = 64;    // slots per allocation (3 MiB)
constexpr int kSlotReserve = 32;  // free slots kept for graph captures

static int grow_pool(int d, SlotPool &p) {  // p.mu held; the caller's stream is not capturing
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess) return set_error(KVECC_ENODEV, "hipGetDevice failed");
  if (hipSetDevice(d) != hipSuccess) return set_error(KVECC_ENODEV, "hipSetDevice(%d) failed", d);
  hipError_t e = hipSuccess;
  // another stream may be capturing in global mode (torch.cuda.graph's
  // default), which prohibits hipMalloc and stream syncs from every thread in
  // global / thread-local mode and would invalidate that capture: this
  // thread allocates in relaxed mode, then restores its mode
  hipStreamCaptureMode mode = hipStreamCaptureModeRelaxed;
  const bool exchanged = hipThreadExchangeStreamCaptureMode(&mode) == hipSuccess;
  {
    uint32_t *mem = nullptr;
    const size_t bytes = sizeof(uint32_t) * (size_t)kSlotChunk * kSlotWords;
    if (!p.side) e = hipStreamCreateWithFlags(&p.side, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&mem, bytes);
    if (e == hipSuccess) e = hipMemsetAsync(mem, 0, bytes, p.side);
    if (e == hipSuccess) e = hipStreamSynchronize(p.side);
    if (e == hipSuccess) {
      p.chunks.push_back(mem);
      for (int i = kSlotChunk - 1; i >= 0; --i) p.free.push_back(mem + (size_t)i * kSlotWords);
    }
  }
  if (exchanged) (void)hipThreadExchangeStreamCaptureMode(&mode);
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return set_error(KVECC_EHIP, "counter slots: %s", hipGetErrorString(e));
  return KVECC_OK;
}

// slots whose graphs are gone: back to the free list (p.mu held)
static void drain_returned(SlotPool &p) {
  std::vector<uint32_t *> back;
  {
    std::lock_guard<std::mutex> lk(p.ret_mu);
    back.swap(p.returned);
  }
  for (uint32_t *s : back) {
    for (auto it = p.captured.begin(); it != p.captured.end();)
      it = it->second == s ? p.captured.erase(it) : std::next(it);
    p.free.push_back(s);
  }
}

struct SlotRelease {
  int dev;
  uint32_t *slot;
};

static void release_captured_slot(void *arg) {  // HIP user-object destructor
  SlotRelease *r = static_cast<SlotRelease *>(arg);
  if (r->slot) {  // null: the slot was never tied to a graph and stays with its capture
    SlotPool &p = g_pool[r->dev];
    std::lock_guard<std::mutex> lk(p.ret_mu);
    p.returned.push_back(r->slot);
  }
  delete r;
}

static int ensure_pool(int d) {
  if (d < 0 || d >= kMaxDev) return set_error(KVECC_EINVAL, "device %d out of range", d);
  SlotPool &p = g_pool[d];
  std::lock_guard<std::mutex> lk(p.mu);
  return p.chunks.empty() ? grow_pool(d, p) : KVECC_OK;
}

uint32_t *counter_slot(void *stream) {
  const int d = current_device();
  if (d < 0 || d >= kMaxDev) {
    set_error(KVECC_EINVAL, "device %d out of range", d);
    return nullptr;
  }
  hipStream_t st = as_stream(stream);
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  unsigned long long cid = 0;
  hipGraph_t graph = nullptr;
  if (hipStreamGetCaptureInfo_v2(st, &cs, &cid, &graph, nullptr, nullptr) != hipSuccess)
    cs = hipStreamCaptureStatusNone;
  uint64_t key = reinterpret_cast<uint64_t>(stream);
  if (st == hipStreamPerThread)  // one handle, a different stream in every thread
    key = (uint64_t)std::hash<std::thread::id>{}(std::this_thread::get_id()) | (1ull << 63);
  SlotPool &p = g_pool[d];
  std::lock_guard<std::mutex> lk(p.mu);
  drain_returned(p);
  const bool capturing = cs == hipStreamCaptureStatusActive;
  if (!capturing) {
    // keep the reserve for captures topped up (allocation is illegal during one).
    // The reserve is a target: when growth fails -- e.g. another stream is
    // capturing in global mode, which forbids hipMalloc from every thread -- an
    // eager launch still takes a free slot, and the failed call's error is
    // consumed so the launch does not report it
    if (p.free.size() <= (size_t)kSlotReserve && grow_pool(d, p) != KVECC_OK) {
      (void)hipGetLastError();
      if (p.free.empty()) return nullptr;
    }
    auto it = p.eager.find(key);
    if (it != p.eager.end()) return it->second;
    uint32_t *s = p.free.back();
    p.free.pop_back();
    p.eager.emplace(key, s);
    return s;
  }
  auto it = p.captured.find({key, cid});
  if (it != p.captured.end()) return it->second;
  if (p.free.empty()) {
    set_error(KVECC_EHIP,
              "no free counter slot during graph capture (call kvecc_reserve_counter_slots before capturing)");
    return nullptr;
  }
  uint32_t *s = p.free.back();
  p.free.pop_back();
  // a stream is in one capture at a time: its earlier captures' entries are done
  for (auto jt = p.captured.begin(); jt != p.captured.end();)
    jt = jt->first.first == key ? p.captured.erase(jt) : std::next(jt);
  p.captured.emplace(std::make_pair(key, cid), s);
  // tie the slot to the graph; without a graph handle or user objects it stays
  // allocated for the process (the pre-round-5 behaviour)
  if (graph) {
    SlotRelease *r = new SlotRelease{d, s};
    hipUserObject_t obj = nullptr;
    if (hipUserObjectCreate(&obj, r, release_captured_slot, 1, hipUserObjectNoDestructorSync) != hipSuccess) {
      delete r;
    } else if (g_fail_retain.load(std::memory_order_relaxed) ||
               hipGraphRetainUserObject(graph, obj, 1, hipGraphUserObjectMove) != hipSuccess) {
      // the graph does not hold the object, so nothing tells us when the graph
      // dies: the slot must stay with this capture for the process's life (as
      // with no graph handle).  Detach it before dropping our reference, whose
      // destructor would otherwise return a slot the capture still uses
      r->slot = nullptr;
      (void)hipUserObjectRelease(obj, 1);
      (void)hipGetLastError();
    }
  }
  return s;
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
  const int rc = ensure_tables(device);
  return rc != KVECC_OK ? rc : ensure_pool(device);
}

KVECC_API int kvecc_reserve_counter_slots(int device, int n) {
  int nd = kvecc_device_count();
  if (nd <= 0) return set_error(KVECC_ENODEV, "no HIP device visible");
  if (device < 0 || device >= nd || device >= kMaxDev || n < 0)
    return set_error(KVECC_EINVAL, "reserve_counter_slots: bad device %d or count %d", device, n);
  SlotPool &p = g_pool[device];
  std::lock_guard<std::mutex> lk(p.mu);
  drain_returned(p);
  while (p.free.size() < (size_t)n + kSlotReserve) {
    const int rc = grow_pool(device, p);
    if (rc != KVECC_OK) return rc;
  }
  return KVECC_OK;
}

KVECC_API int kvecc_debug_fail_graph_retain(int on) {
  g_fail_retain.store(on ? 1 : 0, std::memory_order_relaxed);
  return KVECC_OK;
}

KVECC_API int kvecc_counter_slots_check(int device, int64_t *slots_in_use, int64_t *nonzero_words) {
  int nd = kvecc_device_count();
  if (nd <= 0) return set_error(KVECC_ENODEV, "no HIP device visible");
  if (device < 0 || device >= nd || device >= kMaxDev || !slots_in_use || !nonzero_words)
    return set_error(KVECC_EINVAL, "counter_slots_check: bad argument");
  SlotPool &p = g_pool[device];
  std::lock_guard<std::mutex> lk(p.mu);
  drain_returned(p);
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess)
    return set_error(KVECC_ENODEV, "hipSetDevice(%d) failed", device);
  hipError_t e = hipDeviceSynchronize();
  std::vector<uint32_t> h((size_t)kSlotChunk * kSlotWords);
  int64_t nz = 0;
  for (uint32_t *c : p.chunks) {
    if (e == hipSuccess) e = hipMemcpy(h.data(), c, h.size() * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (e != hipSuccess) break;
    for (uint32_t v : h) nz += v != 0;
  }
  (void)hipSetDevice(prev);
  if (e != hipSuccess) return set_error(KVECC_EHIP, "counter_slots_check: %s", hipGetErrorString(e));
  *slots_in_use = (int64_t)(p.chunks.size() * kSlotChunk - p.free.size());
  *nonzero_words = nz;
  return KVECC_OK;
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
