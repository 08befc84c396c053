// pg_runtime.hip -- libpinot_gpu host runtime: device binding, segment residency, plan compilation,
// launch sequencing and result decoding behind the C ABI of include/pinot_gpu.h.
//
// Mirrors on the device side what the reference does per query on the server:
//   InstancePlanMakerImplV2.makeInstancePlan (plan/maker/InstancePlanMakerImplV2.java:153-187)
//     -> per segment FilterPlanNode.constructPhysicalOperator (plan/FilterPlanNode.java:191-311)
//        choosing scan / sorted / inverted leaves (operator/filter/FilterOperatorUtils.java:45-85)
//     -> AggregationOperator / AggregationGroupByOrderByOperator
//     -> AggregationOnlyCombineOperator / GroupByOrderByCombineOperator merge
// but as ONE fused launch over all of the query's segments on this GPU (plus a small pre-pass for
// index-backed leaves), with per-group state merged in device memory by global key id.
#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <sched.h>
#include <signal.h>
#include <unistd.h>
#include <time.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <deque>
#include <functional>
#include <future>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "pg_aux.h"
#include "../../include/pinot_codec.h"
#include "../../include/pinot_trace.h"

using namespace pg;

namespace {

thread_local std::string t_err;
thread_local pg_timing t_timing{};
thread_local pg_trace t_trace{};  // pg_last_trace: the calling thread's last device call (pinot_trace.h)
int g_device = -1;                // HIP device of logical device 0 (pg_init / pg_init_devices)
std::mutex g_init_mu;
// Logical devices (pg_init_devices): logical device i runs on HIP device g_ldev_phys[i]; a device may repeat (two
// logical devices sharing one GPU, each with its own worker thread and stream).  One entry for pg_init.
constexpr int kMaxPhys = 64;
std::vector<int> g_ldev_phys;
thread_local int t_ldev = 0;      // the logical device this thread works for (a worker's own; 0 for caller threads)
int cur_phys() {                  // the HIP device this thread's device work goes to
  return g_ldev_phys.empty() ? std::max(g_device, 0) : g_ldev_phys[(size_t)t_ldev < g_ldev_phys.size() ? t_ldev : 0];
}

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  return code;
}

#define HIP_CHECK(expr)                                                                                  \
  do {                                                                                                   \
    hipError_t _e = (expr);                                                                              \
    if (_e != hipSuccess) return fail(PG_E_HIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),   \
                                      __FILE__, __LINE__);                                               \
  } while (0)

int ensure_device() {
  if (g_device < 0) return fail(PG_E_STATE, "pg_init has not been called");
  const int dev = cur_phys();
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != dev) {
    if (hipSetDevice(dev) != hipSuccess) return fail(PG_E_HIP, "hipSetDevice(%d) failed", dev);
  }
  return PG_OK;
}

hipStream_t thread_stream() {
  thread_local hipStream_t s = nullptr;
  if (!s) hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  return s;
}

double wall_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

// Host-side phase profile of one query (PG_HOST_PROFILE=1: printed to stderr after each execute; dev tool).
struct HostProf {
  const char* name[32];
  double t[32];
  int n = 0;
};
thread_local HostProf t_prof;
bool host_prof_on() {
  static const bool on = getenv("PG_HOST_PROFILE") && atoi(getenv("PG_HOST_PROFILE")) != 0;
  return on;
}
#define PG_PROF(label) \
  do { if (host_prof_on() && t_prof.n < 32) { t_prof.name[t_prof.n] = label; t_prof.t[t_prof.n++] = wall_ms(); } } while (0)
void host_prof_dump(double t0) {
  if (!host_prof_on()) return;
  double prev = t0;
  fprintf(stderr, "[pg host]");
  for (int i = 0; i < t_prof.n; i++) { fprintf(stderr, " %s=%.1fus", t_prof.name[i], (t_prof.t[i] - prev) * 1e3); prev = t_prof.t[i]; }
  fprintf(stderr, " total=%.1fus\n", (prev - t0) * 1e3);
  t_prof.n = 0;
}

int64_t now_ms() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (int64_t)ts.tv_sec * 1000 + ts.tv_nsec / 1000000;
}

// ------------------------------------------------------------------------------------------ residency

// Caching device allocator for per-query buffers (parameter arena, filter scratch, partial state):
// power-of-two buckets, hipMalloc on a miss, blocks parked for reuse instead of freed, so steady-state queries
// make no hipMalloc / hipFree calls.  A block is returned only after the host has synchronised with every
// launch that used it.
class DevicePool {
 public:
  void* get(uint64_t bytes, uint64_t* cap) {
    uint64_t c = 256;
    while (c < bytes) c <<= 1;
    *cap = c;
    {
      std::lock_guard<std::mutex> g(mu_);
      auto& v = free_[c];
      if (!v.empty()) {
        void* p = v.back();
        v.pop_back();
        return p;
      }
    }
    void* p = nullptr;
    if (hipMalloc(&p, c) != hipSuccess) return nullptr;
    return p;
  }
  void put(void* p, uint64_t cap) {
    std::lock_guard<std::mutex> g(mu_);
    free_[cap].push_back(p);
  }

 private:
  std::mutex mu_;
  std::unordered_map<uint64_t, std::vector<void*>> free_;
};
DevicePool g_pools[kMaxPhys];  // one per HIP device: a block is only ever reused on the device it was allocated on

// Device buffer: resident index buffers own a hipMalloc allocation; per-query buffers borrow a pool block.
struct DevBuf {
  void* p = nullptr;
  uint64_t bytes = 0;
  uint64_t cap = 0;
  bool pooled = false;
  int pdev = 0;  // pooled: the HIP device (pool) the block came from
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept { *this = std::move(o); }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      reset();
      p = o.p; bytes = o.bytes; cap = o.cap; pooled = o.pooled; pdev = o.pdev;
      o.p = nullptr; o.bytes = 0; o.cap = 0;
    }
    return *this;
  }
  ~DevBuf() { reset(); }
  void reset() {
    if (p) {
      if (pooled) g_pools[pdev].put(p, cap);
      else (void)hipFree(p);
    }
    p = nullptr;
    bytes = cap = 0;
  }
  int alloc(uint64_t n) {
    reset();
    if (n == 0) n = 16;
    pooled = false;
    if (hipMalloc(&p, n) != hipSuccess) {
      p = nullptr;
      return fail(PG_E_NOMEM, "hipMalloc(%llu) failed", (unsigned long long)n);
    }
    bytes = cap = n;
    return PG_OK;
  }
  int alloc_pooled(uint64_t n) {
    reset();
    if (n == 0) n = 16;
    pooled = true;
    pdev = cur_phys();
    p = g_pools[pdev].get(n, &cap);
    if (!p) return fail(PG_E_NOMEM, "device allocation of %llu bytes failed", (unsigned long long)n);
    bytes = n;
    return PG_OK;
  }
};

// Pinned host staging for the per-query parameter arena (one H2D DMA, no pageable bounce).
// Fine-grained and mapped (`dp`: the device's address of p), so a kernel can write it directly (launch_copy_spans).
struct PinnedBuf {
  void* p = nullptr;
  void* dp = nullptr;
  uint64_t cap = 0;
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
  void* get(uint64_t n) {
    if (n > cap) {
      if (p) (void)hipHostFree(p);
      p = dp = nullptr;
      cap = 1;
      while (cap < n) cap <<= 1;
      if (hipHostMalloc(&p, cap, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !p ||
          hipHostGetDevicePointer(&dp, p, 0) != hipSuccess || !dp) {
        if (p) (void)hipHostFree(p);
        p = dp = nullptr;
        cap = 0;
      }
    }
    return p;
  }
  void* dev(const void* host) const { return (uint8_t*)dp + ((const uint8_t*)host - (const uint8_t*)p); }
};

// Growable pinned host buffer whose capacity persists across queries: the parameter arena is built in it directly and
// copied to the device from it (no staging memcpy).
struct PinnedVec {
  uint8_t* p = nullptr;
  void* dp = nullptr;  // the device's address of p
  uint64_t n = 0, cap = 0;
  ~PinnedVec() {
    if (p) (void)hipHostFree(p);
  }
  uint64_t size() const { return n; }
  uint8_t* data() { return p; }
  uint8_t& operator[](uint64_t i) { return p[i]; }
  void clear() { n = 0; }
  void grow(uint64_t m) {  // size m, contents [0, n) kept
    if (m > cap) {
      uint64_t c = cap ? cap : 4096;
      while (c < m) c <<= 1;
      void* q = nullptr;
      // fine-grained and mapped: the device reads it directly (launch_arena_upload), never a stale cached line
      if (hipHostMalloc(&q, c, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess || !q) throw std::bad_alloc();
      void* d = nullptr;
      if (hipHostGetDevicePointer(&d, q, 0) != hipSuccess || !d) {
        (void)hipHostFree(q);
        throw std::bad_alloc();
      }
      if (n) memcpy(q, p, n);
      if (p) (void)hipHostFree(p);
      p = (uint8_t*)q;
      dp = d;
      cap = c;
    }
    n = m;
  }
};

enum FwdKind : uint32_t { FWD_NONE = 0, FWD_SV = 1, FWD_SORTED = 2, FWD_MV = 3, FWD_RAW = 4 };

struct ColumnRes {
  // dictionary
  bool has_dict = false;
  uint32_t dtype = 0, card = 0, entry_bytes = 0;
  DevBuf dict;
  double dmin = 0, dmax = 0;  // dictionary min / max value (as double; integers exact below 2^53)
  int64_t imin = 0, imax = 0;
  double fin_abs = 0;         // largest |value| among the finite values (the SK_FX windows' upper bound)
  double fin_min = 0;         // smallest nonzero |value| among the finite values, 0 = none (their lower bound)
  bool nonfinite = false;     // some value is +-inf or NaN (FLOAT / DOUBLE)
  // forward index
  uint32_t fwd = FWD_NONE;
  uint32_t num_docs = 0, bits = 0, num_values = 0;
  DevBuf words;                       // packed dictIds (SV / synthesised for sorted / MV values)
  DevBuf mv_offsets;                  // MV row offsets
  DevBuf mv_cnt;                      // MV values per doc, 4-bit packed (absent when a doc holds more than 15)
  std::vector<int32_t> sorted_pairs;  // host copy for leaf lowering (card x 2)
  // inverted index
  bool has_inv = false;
  DevBuf roaring, containers, inv_dir_dev;
  std::vector<uint32_t> inv_dir;  // CSR: containers of dictId d are [inv_dir[d], inv_dir[d+1]) (+ a device copy)
  DevBuf inv_keydir;              // key-major: [key * card + dictId] = keydir_entry of the container (when small enough)
  uint32_t inv_keydir_card = 0;
  // keymap
  bool has_keymap = false;
  DevBuf keymap;
  // decoded forward index (value - imin, vbits bits per doc) of a large INT / LONG dictionary, built once both the
  // dictionary and the SV forward index are resident (launch_decode_pack); read by group keys and aggregation
  // inputs in place of dictId + dictionary gather
  DevBuf vals;
  uint32_t vbits = 0;
  // raw (no-dictionary) forward index: the num_docs values, native typed (dtype), decoded from the chunks at upload
  DevBuf rawv;
  // range index (PG_IDX_RANGE): present; a raw INT / LONG column's device form is `vals` (value - imin, vbits bits)
  bool has_range = false;
  // identity dictionary: INT / LONG values imin, imin + 1, ..., imin + card - 1 (every value of a dense range present),
  // so value = imin + dictId and the packed dictIds serve as the decoded forward index (no dictionary reads)
  bool identity = false;
};

// Dictionaries at least this large get a decoded forward index (PG_DECODED=0 disables, =1 builds it for every
// INT / LONG dictionary): below it the dictionary stays cache-resident and the gather is cheap.
constexpr uint32_t kDecodeMinCard = 1u << 17;
// key-major roaring container directories up to this many entries per column (64 M entries = 256 MB)
constexpr uint64_t kKeyDirMaxEntries = 1ull << 26;

// Build c.vals when c has an INT / LONG dictionary of >= kDecodeMinCard values and an SV bit-packed forward index.
int build_decoded(ColumnRes& c, hipStream_t s) {
  static const char* env = getenv("PG_DECODED");
  const int mode = env ? atoi(env) : -1;
  c.vals.reset();
  c.vbits = 0;
  c.identity = mode != 0 && c.has_dict && c.fwd == FWD_SV && (c.dtype == PG_INT || c.dtype == PG_LONG) && c.card &&
               c.imax >= c.imin && (uint64_t)(c.imax - c.imin) + 1 == (uint64_t)c.card;
  if (c.identity) return PG_OK;
  if (mode == 0 || !c.has_dict || c.fwd != FWD_SV || (c.dtype != PG_INT && c.dtype != PG_LONG) || !c.card ||
      !c.num_docs || (mode != 1 && c.card < kDecodeMinCard))
    return PG_OK;
  const uint64_t span = (uint64_t)(c.imax - c.imin);
  if (c.imax < c.imin || span >= (1ull << 32)) return PG_OK;
  uint32_t vb = 1;
  while (vb < 32 && (span >> vb)) vb++;
  const uint64_t nwords = ((uint64_t)c.num_docs * vb + 31) / 32 + 4;
  int rc;
  if ((rc = c.vals.alloc(nwords * 4))) return rc;
  HIP_CHECK(launch_decode_pack((const uint32_t*)c.words.p, c.bits, c.dict.p, c.dtype, c.card, c.imin, vb, c.num_docs,
                               (uint32_t*)c.vals.p, nwords, s));
  HIP_CHECK(hipStreamSynchronize(s));
  c.vbits = vb;
  return PG_OK;
}

struct SegmentRes {
  std::unordered_map<uint32_t, ColumnRes> cols;
  uint32_t ldev = 0;  // the logical device holding it (pg_init_devices / pg_segment_place)
};

std::shared_mutex g_seg_mu;
std::unordered_map<uint64_t, SegmentRes*> g_segs;
std::mutex g_cancel_mu;
std::unordered_set<uint64_t> g_cancelled;

bool is_cancelled(uint64_t qid) {
  if (!qid) return false;
  std::lock_guard<std::mutex> g(g_cancel_mu);
  return g_cancelled.count(qid) != 0;
}

// In-flight cancellation: a slot of host-coherent pinned flags per running cancellable query (query_id or deadline),
// polled by the scan kernel once per tile.  pg_cancel sets 1 (-> PG_E_CANCELLED); the executing thread sets 2 when the
// deadline passes while it waits (-> PG_E_TIMEOUT).  Mirrors BaseOperator.nextBlock's interrupt check
// (operator/BaseOperator.java:35-37) and the QueryContext deadline, at tile granularity inside the one launch.
constexpr uint32_t kCancelSlots = 256;
volatile uint32_t* g_flags = nullptr;        // [kCancelSlots], hipHostMalloc coherent + mapped
std::vector<uint32_t> g_free_slots;           // under g_cancel_mu
std::unordered_multimap<uint64_t, uint32_t> g_inflight;  // query_id -> slot, under g_cancel_mu

struct CancelSlot {
  int slot = -1;
  uint64_t qid = 0;
  CancelSlot(uint64_t q, bool want) : qid(q) {
    if (!want || !g_flags) return;
    std::lock_guard<std::mutex> g(g_cancel_mu);
    if (g_free_slots.empty()) return;  // every slot busy: this query is only checked before launch
    slot = (int)g_free_slots.back();
    g_free_slots.pop_back();
    g_flags[slot] = g_cancelled.count(qid) ? 1u : 0u;
    if (qid) g_inflight.emplace(qid, (uint32_t)slot);
  }
  ~CancelSlot() {
    if (slot < 0) return;
    std::lock_guard<std::mutex> g(g_cancel_mu);
    auto r = g_inflight.equal_range(qid);
    for (auto it = r.first; it != r.second; ++it)
      if (it->second == (uint32_t)slot) { g_inflight.erase(it); break; }
    g_free_slots.push_back((uint32_t)slot);
  }
  const unsigned int* device_ptr() const { return slot < 0 ? nullptr : (const unsigned int*)(g_flags + slot); }
  uint32_t state() const { return slot < 0 ? 0u : g_flags[slot]; }
  void set(uint32_t v) { if (slot >= 0 && g_flags[slot] == 0) g_flags[slot] = v; }
};

int init_cancel_flags() {  // under g_init_mu
  if (g_flags) return PG_OK;
  void* p = nullptr;
  HIP_CHECK(hipHostMalloc(&p, kCancelSlots * 4, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable));
  memset(p, 0, kCancelSlots * 4);
  std::lock_guard<std::mutex> g(g_cancel_mu);
  for (uint32_t i = 0; i < kCancelSlots; i++) g_free_slots.push_back(kCancelSlots - 1 - i);
  g_flags = (volatile uint32_t*)p;
  return PG_OK;
}

inline uint32_t rd_be32(const uint8_t* p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}
inline uint64_t rd_be64(const uint8_t* p) { return ((uint64_t)rd_be32(p) << 32) | rd_be32(p + 4); }
inline uint16_t rd_le16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
inline uint32_t rd_le32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

double be_value_as_double(const uint8_t* p, uint32_t dtype) {
  switch (dtype) {
    case PG_INT: return (double)(int32_t)rd_be32(p);
    case PG_LONG: return (double)(int64_t)rd_be64(p);
    case PG_FLOAT: { uint32_t u = rd_be32(p); float f; memcpy(&f, &u, 4); return f; }
    case PG_DOUBLE: { uint64_t u = rd_be64(p); double d; memcpy(&d, &u, 8); return d; }
    default: return 0;
  }
}
int64_t be_value_as_i64(const uint8_t* p, uint32_t dtype) {
  return dtype == PG_INT ? (int64_t)(int32_t)rd_be32(p) : (dtype == PG_LONG ? (int64_t)rd_be64(p) : 0);
}

// Copy `src` (host or device) into a fresh device staging buffer.
int stage(const void* src, uint64_t nbytes, bool src_device, DevBuf& out, hipStream_t s) {
  int rc = out.alloc(nbytes + 16);
  if (rc) return rc;
  HIP_CHECK(hipMemsetAsync(out.p, 0, nbytes + 16, s));
  if (nbytes)
    HIP_CHECK(hipMemcpyAsync(out.p, src, nbytes, src_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
  return PG_OK;
}

// Host copy of a (host or device) source range.
int host_copy(const void* src, uint64_t nbytes, bool src_device, std::vector<uint8_t>& out) {
  out.resize(nbytes);
  if (!nbytes) return PG_OK;
  if (src_device) HIP_CHECK(hipMemcpy(out.data(), src, nbytes, hipMemcpyDeviceToHost));
  else memcpy(out.data(), src, nbytes);
  return PG_OK;
}

// Parse a BitmapInvertedIndexWriter buffer: (card+1) BE uint32 offsets + portable roarings
// (readers/BitmapInvertedIndexReader.java:45-63); re-lay every container payload 8-byte aligned.
int parse_inverted(const std::vector<uint8_t>& b, uint32_t card, std::vector<uint32_t>& dir,
                   std::vector<RoaringContainer>& cs, std::vector<uint8_t>& payload) {
  if (b.size() < 4ull * (card + 1)) return fail(PG_E_INVALID, "inverted index too small");
  const uint64_t base = 4ull * (card + 1);
  const uint32_t first = rd_be32(&b[0]);
  dir.assign(card + 1, 0);
  for (uint32_t d = 0; d < card; d++) {
    dir[d] = (uint32_t)cs.size();
    const uint64_t s = base + (uint64_t)(rd_be32(&b[4ull * d]) - first);
    const uint64_t e = base + (uint64_t)(rd_be32(&b[4ull * (d + 1)]) - first);
    if (e > b.size() || s > e || e - s < 8) return fail(PG_E_INVALID, "bad roaring offsets for dictId %u", d);
    const uint8_t* r = &b[s];
    const uint32_t cookie = rd_le32(r);
    uint32_t size, pos;
    const uint8_t* run_flags = nullptr;
    if ((cookie & 0xFFFF) == 12347) {
      size = (cookie >> 16) + 1;
      pos = 4;
      run_flags = r + pos;
      pos += (size + 7) / 8;
    } else if (cookie == 12346) {
      size = rd_le32(r + 4);
      pos = 8;
    } else {
      return fail(PG_E_INVALID, "bad roaring cookie %u for dictId %u", cookie, d);
    }
    const uint32_t hdr = pos;
    pos += 4 * size;
    const bool has_off = !run_flags || size >= 4;
    const uint32_t off_pos = pos;
    if (has_off) pos += 4 * size;
    uint32_t cur = pos;
    for (uint32_t i = 0; i < size; i++) {
      RoaringContainer c;
      c.key = rd_le16(r + hdr + 4 * i);
      const uint32_t cardm1 = rd_le16(r + hdr + 4 * i + 2);
      if (has_off) cur = rd_le32(r + off_pos + 4 * i);
      const bool is_run = run_flags && ((run_flags[i / 8] >> (i % 8)) & 1);
      uint32_t len;
      if (is_run) {
        c.type = 2;
        c.card = rd_le16(r + cur);
        len = 2 + 4 * c.card;
      } else if (cardm1 + 1 <= 4096) {
        c.type = 0;
        c.card = cardm1 + 1;
        len = 2 * c.card;
      } else {
        c.type = 1;
        c.card = cardm1 + 1;
        len = 8192;
      }
      if (s + cur + len > e) return fail(PG_E_INVALID, "roaring container overruns dictId %u", d);
      const uint64_t at = (payload.size() + 7) & ~7ull;
      payload.resize(at + len);
      memcpy(&payload[at], r + cur, len);
      c.offset = (uint32_t)at;
      cs.push_back(c);
      cur += len;
    }
  }
  dir[card] = (uint32_t)cs.size();
  // payloads re-laid key-major (by 64 K-doc key, then dictId): a key's decode reads the selected dictIds' containers
  // of that key from one contiguous region instead of one scattered line per container
  std::vector<uint32_t> order(cs.size());
  for (uint32_t i = 0; i < (uint32_t)cs.size(); i++) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return cs[x].key < cs[y].key; });
  std::vector<uint8_t> km;
  km.reserve(payload.size() + 8);
  for (uint32_t i : order) {
    RoaringContainer& c = cs[i];
    const uint64_t len = c.type == 0 ? 2ull * c.card : (c.type == 1 ? 8192ull : 2ull + 4ull * c.card);
    const uint64_t at = (km.size() + 7) & ~7ull;
    if (at + len > 0xFFFFFFFFull) return fail(PG_E_UNSUPPORTED, "inverted index payload past 4 GiB");
    km.resize(at + len);
    memcpy(&km[at], &payload[c.offset], len);
    c.offset = (uint32_t)at;
  }
  km.resize((km.size() + 7) & ~7ull);  // whole 8-byte words: the device reads array entries 4 at a time
  payload.swap(km);
  return PG_OK;
}

// A raw chunked forward index (BaseChunkForwardIndexReader.java:56-102 header; FixedByteChunkSVForwardIndexReader /
// FixedBytePower2ChunkSVForwardIndexReader per-doc reads) -> the big-endian values of docs [0, num_docs).
int raw_forward_values(const std::vector<uint8_t>& b, uint32_t width, uint32_t num_docs, std::vector<uint8_t>& out) {
  if (b.size() < 16) return fail(PG_E_INVALID, "raw forward index: %zu-byte header", b.size());
  const uint32_t version = rd_be32(&b[0]), num_chunks = rd_be32(&b[4]), per_chunk = rd_be32(&b[8]), entry = rd_be32(&b[12]);
  if (entry != width) return fail(PG_E_INVALID, "raw forward index: entry size %u != %u", entry, width);
  uint32_t comp = 1 /* SNAPPY */, data_start = 16;
  if (version > 1) {
    if (b.size() < 28) return fail(PG_E_INVALID, "raw forward index: short v%u header", version);
    comp = rd_be32(&b[20]);
    data_start = rd_be32(&b[24]);
  }
  if (version < 1 || version > 4) return fail(PG_E_UNSUPPORTED, "raw forward index version %u", version);
  const uint32_t osz = version <= 2 ? 4 : 8;
  const uint64_t raw_start = (uint64_t)data_start + (uint64_t)num_chunks * osz;
  if (raw_start > b.size()) return fail(PG_E_INVALID, "raw forward index: chunk table past the buffer");
  out.assign((uint64_t)num_docs * width, 0);
  if (comp == 0) {  // PASS_THROUGH: the chunks are the contiguous values
    if (raw_start + out.size() > b.size()) return fail(PG_E_INVALID, "raw forward index: %u docs past the buffer", num_docs);
    memcpy(out.data(), &b[raw_start], out.size());
    return PG_OK;
  }
  if (comp > PG_CODEC_LZ4_LENGTH_PREFIXED) return fail(PG_E_UNSUPPORTED, "raw forward index: chunk compression %u", comp);
  std::vector<uint8_t> chunk((uint64_t)per_chunk * width + 16);
  uint64_t at = 0;
  for (uint32_t k = 0; k < num_chunks && at < out.size(); k++) {
    auto off = [&](uint32_t i) -> uint64_t {
      const uint8_t* q = &b[data_start + (uint64_t)i * osz];
      return osz == 4 ? rd_be32(q) : ((uint64_t)rd_be32(q) << 32) | rd_be32(q + 4);
    };
    const uint64_t s0 = off(k), e0 = k + 1 < num_chunks ? off(k + 1) : b.size();
    if (s0 > e0 || e0 > b.size()) return fail(PG_E_INVALID, "raw forward index: bad chunk %u", k);
    // ChunkDecompressor.decompress of the chunk's codec (pg_codec.hip): at most docsPerChunk entries
    uint64_t got = 0;
    const char* why = "";
    int rc = decompress_chunk(comp, &b[s0], e0 - s0, chunk.data(), (uint64_t)per_chunk * width, &got, &why);
    if (rc) return fail(rc, "raw forward index chunk %u: %s", k, why);
    const uint64_t take = std::min<uint64_t>(got, out.size() - at);
    if (got < std::min<uint64_t>((uint64_t)per_chunk * width, out.size() - at))
      return fail(PG_E_INVALID, "raw forward index: chunk %u holds %llu bytes", k, (unsigned long long)got);
    memcpy(&out[at], chunk.data(), take);
    at += take;
  }
  if (at < out.size()) return fail(PG_E_INVALID, "raw forward index: %llu of %u docs", (unsigned long long)(at / width), num_docs);
  return PG_OK;
}

int upload_column(uint64_t seg_key, uint32_t col_id, const pg_col_desc* d, const void* src, uint64_t nbytes) {
  const bool on_dev = (d->flags & PG_SRC_DEVICE) != 0;
  hipStream_t s = thread_stream();
  ColumnRes tmp;
  DevBuf st;
  int rc = PG_OK;
  // Fill a fresh ColumnRes part, then swap it into the registry under the lock.
  switch (d->kind) {
    case PG_IDX_DICT: {
      if (d->data_type > PG_BYTES) return fail(PG_E_INVALID, "bad dictionary data type %u", d->data_type);
      const uint32_t w = d->data_type == PG_INT || d->data_type == PG_FLOAT ? 4 :
                         (d->data_type == PG_LONG || d->data_type == PG_DOUBLE ? 8 : d->entry_bytes);
      if ((uint64_t)w * d->cardinality > nbytes)
        return fail(PG_E_INVALID, "dictionary: %llu bytes < card %u x %u", (unsigned long long)nbytes, d->cardinality, w);
      tmp.has_dict = true;
      tmp.dtype = d->data_type;
      tmp.card = d->cardinality;
      tmp.entry_bytes = w;
      if (d->data_type <= PG_DOUBLE && d->cardinality) {
        if ((rc = stage(src, nbytes, on_dev, st, s))) return rc;
        if ((rc = tmp.dict.alloc((uint64_t)w * d->cardinality + 16))) return rc;
        HIP_CHECK(launch_be_to_native((const uint8_t*)st.p, tmp.dict.p, d->cardinality, w, s));
        std::vector<uint8_t> ends;
        std::vector<uint8_t> lo(w), hi(w);
        if (on_dev) {
          HIP_CHECK(hipMemcpy(lo.data(), src, w, hipMemcpyDeviceToHost));
          HIP_CHECK(hipMemcpy(hi.data(), (const uint8_t*)src + (uint64_t)w * (d->cardinality - 1), w, hipMemcpyDeviceToHost));
        } else {
          memcpy(lo.data(), src, w);
          memcpy(hi.data(), (const uint8_t*)src + (uint64_t)w * (d->cardinality - 1), w);
        }
        tmp.dmin = be_value_as_double(lo.data(), d->data_type);
        tmp.dmax = be_value_as_double(hi.data(), d->data_type);
        tmp.imin = be_value_as_i64(lo.data(), d->data_type);
        tmp.imax = be_value_as_i64(hi.data(), d->data_type);
        if (std::isfinite(tmp.dmin) && std::isfinite(tmp.dmax) && d->data_type <= PG_LONG) {
          tmp.fin_abs = std::max(fabs(tmp.dmin), fabs(tmp.dmax));
          tmp.fin_min = tmp.fin_abs > 0 ? 1.0 : 0.0;  // a nonzero integer is at least 1
        } else {  // FLOAT / DOUBLE: the smallest nonzero |value| sits anywhere; +-inf / NaN sort to the ends: scan once
          std::vector<uint8_t> all;
          if ((rc = host_copy(src, (uint64_t)w * d->cardinality, on_dev, all))) return rc;
          for (uint32_t i = 0; i < d->cardinality; i++) {
            const double v = be_value_as_double(&all[(uint64_t)i * w], d->data_type);
            if (std::isfinite(v)) {
              tmp.fin_abs = std::max(tmp.fin_abs, fabs(v));
              if (v != 0 && (tmp.fin_min == 0 || fabs(v) < tmp.fin_min)) tmp.fin_min = fabs(v);
            } else {
              tmp.nonfinite = true;
            }
          }
        }
      }
      break;
    }
    case PG_IDX_FWD_SV_BITPACKED: {
      if (d->bits_per_element < 1 || d->bits_per_element > 32) return fail(PG_E_INVALID, "bad bitsPerElement");
      const uint64_t need = ((uint64_t)d->num_docs * d->bits_per_element + 7) / 8;
      if (nbytes < need) return fail(PG_E_INVALID, "forward index: %llu bytes < %llu", (unsigned long long)nbytes,
                                     (unsigned long long)need);
      tmp.fwd = FWD_SV;
      tmp.num_docs = d->num_docs;
      tmp.bits = d->bits_per_element;
      tmp.card = d->cardinality;
      tmp.num_values = d->num_docs;
      const uint64_t nwords = (need + 3) / 4 + 4;
      if ((rc = stage(src, need, on_dev, st, s))) return rc;
      if ((rc = tmp.words.alloc(nwords * 4))) return rc;
      HIP_CHECK(launch_bswap_words((const uint8_t*)st.p, (uint32_t*)tmp.words.p, need, nwords, s));
      break;
    }
    case PG_IDX_FWD_SV_SORTED: {
      if (nbytes < 8ull * d->cardinality) return fail(PG_E_INVALID, "sorted index too small");
      tmp.fwd = FWD_SORTED;
      tmp.num_docs = d->num_docs;
      tmp.card = d->cardinality;
      tmp.bits = d->bits_per_element ? d->bits_per_element : 1;
      tmp.num_values = d->num_docs;
      std::vector<uint8_t> hb;
      if ((rc = host_copy(src, 8ull * d->cardinality, on_dev, hb))) return rc;
      tmp.sorted_pairs.resize(2ull * d->cardinality);
      for (uint64_t i = 0; i < 2ull * d->cardinality; i++) tmp.sorted_pairs[i] = (int32_t)rd_be32(&hb[4 * i]);
      DevBuf pairs;
      if ((rc = pairs.alloc(8ull * d->cardinality + 16))) return rc;
      HIP_CHECK(hipMemcpyAsync(pairs.p, tmp.sorted_pairs.data(), 8ull * d->cardinality, hipMemcpyHostToDevice, s));
      const uint64_t nwords = ((uint64_t)d->num_docs * tmp.bits + 31) / 32 + 4;
      if ((rc = tmp.words.alloc(nwords * 4))) return rc;
      HIP_CHECK(launch_sorted_to_packed((const int32_t*)pairs.p, d->cardinality, d->num_docs, tmp.bits,
                                        (uint32_t*)tmp.words.p, nwords, s));
      HIP_CHECK(hipStreamSynchronize(s));
      pairs.reset();
      break;
    }
    case PG_IDX_FWD_MV_BITPACKED: {
      const uint32_t nd = d->num_docs, nv = d->num_values, b = d->bits_per_element;
      if (!nd || nv < nd) return fail(PG_E_INVALID, "MV column needs num_values >= num_docs > 0");
      if (b < 1 || b > 32) return fail(PG_E_INVALID, "bad bitsPerElement");
      // FixedBitMVForwardIndexReader.java:61-75
      const uint32_t avg = nv / nd;
      const uint32_t dpc = (uint32_t)ceilf(2048.0f / (float)avg);
      const uint64_t nchunks = (nd + dpc - 1) / dpc;
      const uint64_t hdr = 4 * nchunks, bm_bytes = ((uint64_t)nv + 7) / 8, raw = ((uint64_t)nv * b + 7) / 8;
      if (nbytes < hdr + bm_bytes + raw) return fail(PG_E_INVALID, "MV forward index too small");
      tmp.fwd = FWD_MV;
      tmp.num_docs = nd;
      tmp.num_values = nv;
      tmp.bits = b;
      tmp.card = d->cardinality;
      if ((rc = stage(src, nbytes, on_dev, st, s))) return rc;
      const uint64_t bm_words = (bm_bytes + 3) / 4 + 4, raw_words = (raw + 3) / 4 + 4;
      DevBuf bm;
      if ((rc = bm.alloc(bm_words * 4))) return rc;
      if ((rc = tmp.words.alloc(raw_words * 4))) return rc;
      HIP_CHECK(launch_bswap_words((const uint8_t*)st.p + hdr, (uint32_t*)bm.p, bm_bytes, bm_words, s));
      HIP_CHECK(launch_bswap_words((const uint8_t*)st.p + hdr + bm_bytes, (uint32_t*)tmp.words.p, raw, raw_words, s));
      if ((rc = tmp.mv_offsets.alloc(4ull * (nd + 1)))) return rc;
      DevBuf scratch;
      const size_t sb = mv_offsets_scratch_bytes(nv);
      if ((rc = scratch.alloc(sb))) return rc;
      HIP_CHECK(launch_mv_offsets((const uint32_t*)bm.p, nv, nd, (uint32_t*)tmp.mv_offsets.p, scratch.p, sb, s));
      {  // COUNTMV's 4-bit count column (the fused index count reads 0.5 B per doc instead of two offsets)
        const uint64_t cw = ((uint64_t)nd + 7) / 8 + 4;
        DevBuf over;
        if ((rc = tmp.mv_cnt.alloc(4 * cw)) || (rc = over.alloc(16))) return rc;
        HIP_CHECK(hipMemsetAsync(over.p, 0, 4, s));
        HIP_CHECK(launch_mv_counts((const uint32_t*)tmp.mv_offsets.p, nd, (uint32_t*)tmp.mv_cnt.p, (unsigned int*)over.p, s));
        uint32_t big = 0;
        HIP_CHECK(hipMemcpyAsync(&big, over.p, 4, hipMemcpyDeviceToHost, s));
        HIP_CHECK(hipStreamSynchronize(s));
        if (big) tmp.mv_cnt.reset();  // a doc with more than 15 values: COUNTMV keeps the offsets
      }
      HIP_CHECK(hipStreamSynchronize(s));
      break;
    }
    case PG_IDX_INV_BITMAP: {
      std::vector<uint8_t> hb;
      if ((rc = host_copy(src, nbytes, on_dev, hb))) return rc;
      std::vector<RoaringContainer> cs;
      std::vector<uint8_t> payload;
      if ((rc = parse_inverted(hb, d->cardinality, tmp.inv_dir, cs, payload))) return rc;
      tmp.has_inv = true;
      tmp.card = d->cardinality;
      tmp.num_docs = d->num_docs;
      if ((rc = tmp.roaring.alloc(payload.size() + 16))) return rc;
      if ((rc = tmp.containers.alloc(cs.size() * sizeof(RoaringContainer) + 16))) return rc;
      if (!payload.empty()) HIP_CHECK(hipMemcpyAsync(tmp.roaring.p, payload.data(), payload.size(), hipMemcpyHostToDevice, s));
      if (!cs.empty())
        HIP_CHECK(hipMemcpyAsync(tmp.containers.p, cs.data(), cs.size() * sizeof(RoaringContainer), hipMemcpyHostToDevice, s));
      if ((rc = tmp.inv_dir_dev.alloc(4ull * tmp.inv_dir.size() + 16))) return rc;
      HIP_CHECK(hipMemcpyAsync(tmp.inv_dir_dev.p, tmp.inv_dir.data(), 4ull * tmp.inv_dir.size(), hipMemcpyHostToDevice, s));
      // key-major directory (one load per (dictId, 64 K-doc key) in the pre-pass instead of a binary search over the
      // dictId's containers), kept when it stays within kKeyDirMaxEntries
      const uint64_t nkeys = ((uint64_t)d->num_docs + 65535) >> 16, card = d->cardinality;
      std::vector<uint2> kd;
      if (nkeys * card <= kKeyDirMaxEntries && nkeys * card) {
        kd.assign(nkeys * card, make_uint2(kKeyDirNone, kKeyDirNone));
        for (uint32_t id = 0; id < card; id++)
          for (uint32_t ci = tmp.inv_dir[id]; ci < tmp.inv_dir[id + 1]; ci++)
            if (cs[ci].key < nkeys) kd[(uint64_t)cs[ci].key * card + id] = keydir_entry(cs[ci]);
        if ((rc = tmp.inv_keydir.alloc(8ull * kd.size() + 16))) return rc;
        tmp.inv_keydir_card = (uint32_t)card;
        HIP_CHECK(hipMemcpyAsync(tmp.inv_keydir.p, kd.data(), 8ull * kd.size(), hipMemcpyHostToDevice, s));
      }
      HIP_CHECK(hipStreamSynchronize(s));
      break;
    }
    case PG_IDX_FWD_SV_RAW: {
      if (d->data_type > PG_DOUBLE) return fail(PG_E_UNSUPPORTED, "raw forward index of type %u (fixed-width only)", d->data_type);
      const uint32_t w = d->data_type == PG_INT || d->data_type == PG_FLOAT ? 4 : 8;
      std::vector<uint8_t> hb, be;
      if ((rc = host_copy(src, nbytes, on_dev, hb))) return rc;
      if ((rc = raw_forward_values(hb, w, d->num_docs, be))) return rc;
      tmp.fwd = FWD_RAW;
      tmp.num_docs = d->num_docs;
      tmp.num_values = d->num_docs;
      tmp.dtype = d->data_type;
      tmp.card = d->cardinality;
      // column metadata min / max (ColumnMetadata.getMinValue / getMaxValue): integer-exact SUM bounds, non-scan MIN/MAX
      tmp.dmin = INFINITY;
      tmp.dmax = -INFINITY;
      tmp.imin = INT64_MAX;
      tmp.imax = INT64_MIN;
      for (uint32_t i = 0; i < d->num_docs; i++) {
        const double v = be_value_as_double(&be[(uint64_t)i * w], d->data_type);
        tmp.dmin = std::min(tmp.dmin, v);
        tmp.dmax = std::max(tmp.dmax, v);
        if (std::isfinite(v)) {
          tmp.fin_abs = std::max(tmp.fin_abs, fabs(v));
          if (v != 0 && (tmp.fin_min == 0 || fabs(v) < tmp.fin_min)) tmp.fin_min = fabs(v);
        } else {
          tmp.nonfinite = true;
        }
        if (d->data_type <= PG_LONG) {
          const int64_t x = be_value_as_i64(&be[(uint64_t)i * w], d->data_type);
          tmp.imin = std::min(tmp.imin, x);
          tmp.imax = std::max(tmp.imax, x);
        }
      }
      if ((rc = stage(be.data(), be.size(), false, st, s))) return rc;
      if ((rc = tmp.rawv.alloc((uint64_t)w * d->num_docs + 16))) return rc;
      HIP_CHECK(launch_be_to_native((const uint8_t*)st.p, tmp.rawv.p, d->num_docs, w, s));
      HIP_CHECK(hipStreamSynchronize(s));  // `be` (pageable) is released at the end of this block
      break;
    }
    case PG_IDX_RANGE: {
      // header only (readers/BitSlicedRangeIndexReader.java:44-52, RangeIndexReaderImpl.java:47-95); the body is
      // not needed on the device (see PG_IDX_RANGE in pinot_gpu.h)
      std::vector<uint8_t> hb;
      if ((rc = host_copy(src, std::min<uint64_t>(nbytes, 64), on_dev, hb))) return rc;
      if (hb.size() < 12) return fail(PG_E_INVALID, "range index: %llu bytes", (unsigned long long)nbytes);
      const uint32_t version = rd_be32(&hb[0]);
      if (version == 2) {
        tmp.imin = (int64_t)(((uint64_t)rd_be32(&hb[4]) << 32) | rd_be32(&hb[8]));  // BitSliced min
      } else if (version == 1) {
        const uint32_t len = rd_be32(&hb[4]);
        if (len < 3 || len > 6 || 12 + len > hb.size()) return fail(PG_E_INVALID, "range index v1: bad value type");
        const std::string vt((const char*)&hb[8], len);
        if (vt != "INT" && vt != "LONG" && vt != "FLOAT" && vt != "DOUBLE")
          return fail(PG_E_INVALID, "range index v1: value type %s", vt.c_str());
        tmp.imin = INT64_MIN;  // v1 keeps no min
      } else {
        return fail(PG_E_INVALID, "range index: unknown version %u", version);
      }
      tmp.has_range = true;
      tmp.num_values = version;
      break;
    }
    case PG_IDX_KEYMAP: {
      if (nbytes < 4ull * d->cardinality) return fail(PG_E_INVALID, "keymap too small");
      tmp.has_keymap = true;
      if ((rc = tmp.keymap.alloc(4ull * d->cardinality + 16))) return rc;
      HIP_CHECK(hipMemcpyAsync(tmp.keymap.p, src, 4ull * d->cardinality,
                               on_dev ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s));
      break;
    }
    default:
      return fail(PG_E_INVALID, "unknown index kind %u", d->kind);
  }
  HIP_CHECK(hipStreamSynchronize(s));
  st.reset();

  std::unique_lock<std::shared_mutex> lk(g_seg_mu);
  SegmentRes*& seg = g_segs[seg_key];
  if (!seg) {
    seg = new SegmentRes();
    seg->ldev = (uint32_t)t_ldev;
  }
  ColumnRes& c = seg->cols[col_id];
  switch (d->kind) {
    case PG_IDX_DICT:
      c.dict.reset();
      c.has_dict = true; c.dtype = tmp.dtype; c.card = tmp.card; c.entry_bytes = tmp.entry_bytes;
      c.dict = std::move(tmp.dict);
      c.dmin = tmp.dmin; c.dmax = tmp.dmax; c.imin = tmp.imin; c.imax = tmp.imax;
      c.fin_abs = tmp.fin_abs; c.fin_min = tmp.fin_min; c.nonfinite = tmp.nonfinite;
      break;
    case PG_IDX_FWD_SV_BITPACKED: case PG_IDX_FWD_SV_SORTED: case PG_IDX_FWD_MV_BITPACKED:
      c.words.reset(); c.mv_offsets.reset(); c.mv_cnt.reset();
      c.fwd = tmp.fwd; c.num_docs = tmp.num_docs; c.bits = tmp.bits; c.num_values = tmp.num_values;
      if (!c.has_dict) c.card = tmp.card;
      c.words = std::move(tmp.words);
      c.mv_offsets = std::move(tmp.mv_offsets);
      c.mv_cnt = std::move(tmp.mv_cnt);
      c.sorted_pairs.swap(tmp.sorted_pairs);
      break;
    case PG_IDX_INV_BITMAP:
      c.roaring.reset(); c.containers.reset();
      c.has_inv = true;
      c.roaring = std::move(tmp.roaring);
      c.containers = std::move(tmp.containers);
      c.inv_dir_dev = std::move(tmp.inv_dir_dev);
      c.inv_keydir = std::move(tmp.inv_keydir);
      c.inv_keydir_card = tmp.inv_keydir_card;
      c.inv_dir.swap(tmp.inv_dir);
      if (!c.num_docs) c.num_docs = tmp.num_docs;
      break;
    case PG_IDX_KEYMAP:
      c.keymap.reset();
      c.has_keymap = true;
      c.keymap = std::move(tmp.keymap);
      break;
    case PG_IDX_RANGE: {
      if (c.fwd != FWD_SV && c.fwd != FWD_SORTED && c.fwd != FWD_RAW)
        return fail(PG_E_INVALID, "range index on column %u before its single-value forward index", col_id);
      const bool raw = c.fwd == FWD_RAW;
      // v2 min: 0 for dictIds (BitSlicedRangeIndexCreator.java:46-48), the column min for a raw INT / LONG column
      if (tmp.num_values == 2 && (raw ? (c.dtype <= PG_LONG && tmp.imin != c.imin) : tmp.imin != 0))
        return fail(PG_E_INVALID, "range index min %lld != column %u's", (long long)tmp.imin, col_id);
      c.has_range = true;
      if (raw && c.dtype <= PG_LONG && c.num_docs && c.imax >= c.imin && (uint64_t)(c.imax - c.imin) < (1ull << 30)) {
        uint32_t vb = 1;
        while (vb < 30 && ((uint64_t)(c.imax - c.imin) >> vb)) vb++;
        const uint64_t nwords = ((uint64_t)c.num_docs * vb + 31) / 32 + 4;
        c.vals.reset();
        if ((rc = c.vals.alloc(nwords * 4))) return rc;
        HIP_CHECK(launch_decode_pack(nullptr, 0, c.rawv.p, c.dtype, c.num_docs, c.imin, vb, c.num_docs,
                                     (uint32_t*)c.vals.p, nwords, s));
        HIP_CHECK(hipStreamSynchronize(s));
        c.vbits = vb;
      }
      break;
    }
    case PG_IDX_FWD_SV_RAW:
      c.has_range = false; c.vbits = 0;
      c.words.reset(); c.mv_offsets.reset(); c.mv_cnt.reset(); c.rawv.reset(); c.vals.reset();
      c.fwd = FWD_RAW; c.num_docs = tmp.num_docs; c.bits = 0; c.num_values = tmp.num_values;
      c.dtype = tmp.dtype; c.card = tmp.card; c.has_dict = false;
      c.dmin = tmp.dmin; c.dmax = tmp.dmax; c.imin = tmp.imin; c.imax = tmp.imax;
      c.fin_abs = tmp.fin_abs; c.fin_min = tmp.fin_min; c.nonfinite = tmp.nonfinite;
      c.rawv = std::move(tmp.rawv);
      break;
  }
  if (d->kind == PG_IDX_DICT || d->kind == PG_IDX_FWD_SV_BITPACKED || d->kind == PG_IDX_FWD_SV_SORTED ||
      d->kind == PG_IDX_FWD_MV_BITPACKED)
    return build_decoded(c, s);
  return PG_OK;
}

// ------------------------------------------------------------------------------------------ execution

// ArrayMapBasedHolder state of a wide-key plan (pg_wide.hip): the scan grouped by tuple slot; the tuples map the
// slots back to the K table-global key ids.
struct WideKeys {
  uint32_t K = 0;
  uint64_t cap = 0;
  DevBuf tuples;                       // [cap][K]
  DevBuf tags, misc;                   // a merge target's (pg_partials_create) intern table tags and [fill, err]
  pg_key key1{};                       // the scan's one key: the tuple slot (kWideColId)
  const pg_plan* user_plan = nullptr;  // during finalize: the caller's plan (K keys, its ORDER BY)
};

struct Partials {
  std::shared_ptr<WideKeys> wide;  // set for wide-key plans: packed keys are tuple slots, local to this state
  uint32_t mode = GM_NONE;      // GroupMode (GM_HASH_SEG only between the scan and the truncation merge)
  uint64_t num_slots = 1;
  uint32_t n_i64 = 1, n_fx = 0, n_min = 0, n_max = 0, bit_words = 0, max_fill = 0;
  DevBuf keys, i64, fx, mn, mx, bits, first_doc, misc /* [fill, err] */, seg_matched;
  DevBuf dc_pop;                // GM_PART under pg_execute: each group's DISTINCTCOUNT (aggregation dc_pop_agg)
  int dc_pop_agg = -1;
  bool host_state = false;      // t_ctx.state_host holds a copy of the final state (queued before the scan's sync)
  std::vector<uint32_t> key_card;
  std::vector<uint64_t> key_stride;
  uint32_t projected_cols = 0;
  uint64_t entries_in_filter = 0;
  uint64_t total_docs = 0;
  uint32_t num_segments = 0;
  uint32_t layout = 0;          // bit a: aggregation a accumulates integer-exact (i64) -- must agree across merges
  uint32_t flags = 0;           // PG_RESULT_* seen while producing this state (a segment reached numGroupsLimit)
  std::vector<AggSpec> aggs;
  // signature of the SK_FX units and special slots: states merge only when it agrees (as `layout`)
  uint32_t fx_sig() const {
    uint64_t h = 0x9E3779B97F4A7C15ull;
    for (const AggSpec& a : aggs)
      if (a.kind == SK_FX)
        h = mix64(h ^ ((uint64_t)(uint32_t)a.fx_shift << 32) ^ (a.sp_min != kNoSp ? 1u : 0u) ^ ((uint64_t)a.slot << 8) ^
                  ((uint64_t)a.fx_nwin << 20));
    return (uint32_t)(h >> 33);  // 31 bits: a non-negative int64 in the ranks' fingerprint all-reduce
  }

  StateView view() const {
    StateView v;
    memset(&v, 0, sizeof(v));
    v.num_slots = num_slots;
    v.hmask = mode == GM_HASH || mode == GM_HASH_SEG ? num_slots - 1 : 0;
    v.keys = (unsigned long long*)keys.p;
    v.i64 = (unsigned long long*)i64.p;
    v.fx = (unsigned long long*)fx.p;
    v.mn = (long long*)mn.p;
    v.mx = (long long*)mx.p;
    v.bits = (uint32_t*)bits.p;
    v.first_doc = (unsigned long long*)first_doc.p;
    v.fill = (unsigned int*)misc.p;
    v.err = misc.p ? (unsigned int*)misc.p + 1 : nullptr;
    v.n_i64 = n_i64; v.n_fx = n_fx; v.n_min = n_min; v.n_max = n_max; v.bit_words = bit_words;
    v.max_fill = max_fill;
    v.dc_pop = dc_pop_agg >= 0 ? (const uint32_t*)dc_pop.p : nullptr;
    v.dc_pop_agg = (uint32_t)dc_pop_agg;
    return v;
  }
  // device state for `num_slots` slots of the current layout (+ keys for hash modes), initialised
  int alloc_state(hipStream_t s, bool init = true, FillSpans* defer = nullptr);
};

// Layout of the state arrays of a plan's aggregations (slot assignment, DISTINCTCOUNT bitmap words).  `integer`
// bit a: SUM / AVG a accumulates integer-exact in i64, else exactly as SK_FX in units of 2^fx_shift[a], with special
// slots for non-finite inputs when bit a of `special` is set.
int agg_layout(const pg_plan* plan, uint32_t integer, const std::vector<int32_t>& fx_shift,
               const std::vector<uint32_t>& fx_nwin, uint32_t special, std::vector<AggSpec>& aggs, uint32_t& n_i64,
               uint32_t& n_fx, uint32_t& n_min, uint32_t& n_max, uint32_t& bit_words);

// Pinot's default numGroupsLimit (InstancePlanMakerImplV2.DEFAULT_NUM_GROUPS_LIMIT)
constexpr uint64_t kDefaultNumGroupsLimit = 100000;
constexpr uint64_t kDenseMaxSlots = 1ull << 26;      // dense key spaces up to 64 M slots
constexpr uint64_t kStateBudget = 48ull << 30;       // bytes of group state one query may allocate
constexpr uint64_t kMaxHashSlots = 1ull << 30;
constexpr uint64_t kTrimSelectMinGroups = 1ull << 16;  // ORDER BY trim by radix select from this many groups (else sort)
constexpr uint64_t kPartMinStateBytes = 64ull << 20;  // radix-partitioned group-by above this much dense state

struct PartPlan {  // GM_PART pipeline of one query (pg_part.hip)
  bool on = false;
  uint32_t shift1 = 0, shift2 = 0, vbits = 0, dc_words = 0, dc_word = 0, dc = 0, nparts1 = 0, nparts2 = 1;
};

uint64_t pow2_at_least(uint64_t x) {
  uint64_t c = 1;
  while (c < x) c <<= 1;
  return c;
}

struct Arena {  // host image of the per-query parameter block, copied to the device in one transfer
  PinnedVec& h;  // the calling thread's pinned buffer: its capacity persists, so steady-state queries touch no new pages
  explicit Arena(PinnedVec& buf) : h(buf) { h.clear(); }
  uint64_t put(const void* p, uint64_t n, uint64_t align = 16) {
    uint64_t at = (h.size() + align - 1) & ~(align - 1);
    h.grow(at + n);
    if (n) memcpy(&h[at], p, n);
    return at;
  }
  uint64_t reserve(uint64_t n, uint64_t align = 16) {
    uint64_t at = (h.size() + align - 1) & ~(align - 1);
    h.grow(at + n);
    if (n) memset(&h[at], 0, n);
    return at;
  }
};

struct PrepassOp {  // filter materialisation of an index-backed leaf into a doc bitmap (scratch)
  enum Kind { FILL_RANGES, ROARING, MV_SCAN } kind;
  uint32_t seg, leaf;
  uint64_t in_off = 0;   // arena offset of ranges / selected containers
  uint32_t n = 0;
  uint32_t num_docs = 0;
  uint64_t out_off = 0;  // scratch offset of the doc bitmap
  bool negate = false;
  const ColumnRes* col = nullptr;
  int32_t lo = 0, hi = 0;
  uint64_t lut_off = ~0ull;  // MV scan: scratch LUT offset (or ~0 for a dictId range)
  uint32_t excl = 0;
  uint32_t key0 = 0, nkeys = 0;  // ROARING: the 64 K-doc keys to build (a root-AND doc range bounds them)
};

// ---- filter program: ABI postfix -> tree -> prefix form for the kernel, AND / OR children reordered by
// estimated pass fraction so that later children only see surviving docs (the device analogue of
// FilterOperatorUtils.reorderAndFilterChildOperators, operator/filter/FilterOperatorUtils.java:160-200, plus
// AndDocIdSet evaluating scan children only on the docs the earlier children accepted).
struct FNode {
  int kind;  // 0 leaf, 1 AND, 2 OR, 3 NOT
  int leaf = -1;
  std::vector<int> kids;
  double pass = 1.0;  // estimated fraction of docs accepted
  double cost = 0.0;  // estimated bytes / doc read when evaluated densely
};

int build_tree(const pg_plan* plan, const std::vector<double>& leaf_pass, const std::vector<double>& leaf_cost,
               std::vector<FNode>& nodes, int& root) {
  std::vector<int> st;
  for (uint32_t i = 0; i < plan->num_ops; i++) {
    const int32_t op = plan->ops[i];
    if (op >= 0) {
      FNode n;
      n.kind = 0;
      n.leaf = op;
      n.pass = leaf_pass[op];
      n.cost = leaf_cost[op];
      nodes.push_back(n);
      st.push_back((int)nodes.size() - 1);
    } else if (op == PG_OP_NOT) {
      FNode n;
      n.kind = 3;
      n.kids.push_back(st.back());
      st.pop_back();
      n.pass = 1.0 - nodes[n.kids[0]].pass;
      n.cost = nodes[n.kids[0]].cost;
      nodes.push_back(n);
      st.push_back((int)nodes.size() - 1);
    } else {
      const int cnt = (-op) & 0xFF;
      const int kind = ((-op) & 0x100) ? 1 : 2;
      FNode n;
      n.kind = kind;
      std::vector<int> kids(st.end() - cnt, st.end());
      st.resize(st.size() - cnt);
      for (int k : kids) {  // flatten AND(AND(..)) / OR(OR(..))
        if (nodes[k].kind == kind) n.kids.insert(n.kids.end(), nodes[k].kids.begin(), nodes[k].kids.end());
        else n.kids.push_back(k);
      }
      if (kind == 1) {  // AND: leaves that accept every doc at no cost (match-all, folded into the pre-filter) drop out
        std::vector<int> keep;
        for (int k : n.kids)
          if (!(nodes[k].kind == 0 && nodes[k].pass >= 1.0 && nodes[k].cost <= 0.0)) keep.push_back(k);
        if (keep.empty()) keep.push_back(n.kids[0]);
        n.kids.swap(keep);
      }
      // AND: cheapest-per-rejection first ~ ascending pass fraction, zero-cost leaves (doc ranges, bitmaps)
      // before column scans; OR: descending pass fraction.  Results are order independent.
      auto rank = [&](int k) {
        const double p = kind == 1 ? nodes[k].pass : 1.0 - nodes[k].pass;
        return nodes[k].cost <= 0.0 ? p - 2.0 : p + 1e-3 * nodes[k].cost;
      };
      std::stable_sort(n.kids.begin(), n.kids.end(), [&](int a, int b) { return rank(a) < rank(b); });
      double pass = kind == 1 ? 1.0 : 0.0, cost = 0.0, reach = 1.0;
      for (int k : n.kids) {
        cost += reach * nodes[k].cost;
        if (kind == 1) { pass *= nodes[k].pass; reach = pass; }
        else { pass = 1.0 - (1.0 - pass) * (1.0 - nodes[k].pass); reach = 1.0 - pass; }
      }
      n.pass = pass;
      n.cost = cost;
      nodes.push_back(n);
      st.push_back((int)nodes.size() - 1);
    }
  }
  root = st.empty() ? -1 : st.back();
  return PG_OK;
}

void emit_prefix(const std::vector<FNode>& nodes, int n, std::vector<int32_t>& out) {
  const FNode& x = nodes[n];
  if (x.kind == 0) { out.push_back(x.leaf); return; }
  if (x.kind != 3 && x.kids.size() == 1) { emit_prefix(nodes, x.kids[0], out); return; }
  out.push_back(x.kind == 1 ? kOpAnd : (x.kind == 2 ? kOpOr : kOpNot));
  for (int k : x.kids) emit_prefix(nodes, k, out);
  out.push_back(kOpEnd);
}

// A pre-pass doc bitmap (packed-column bit order) read by the scan as a 1-bit column: doc matches iff bit == 1.
void as_bitmap_leaf(LeafDesc& dl, uint32_t num_docs) {
  dl.kind = LK_RANGE;
  dl.bits = 1;
  dl.lo = 1;
  dl.hi = 2;
  dl.excl = 0;
  dl.wbytes = 4u * ((num_docs + 31) / 32 + 1);
}

// Probability that each leaf is evaluated for a doc (the root's children: 1; an AND child: the product of the
// earlier siblings' pass fractions; an OR child: of their reject fractions).
void assign_reach(const std::vector<FNode>& nodes, int n, double reach, std::vector<double>& leaf_reach) {
  const FNode& x = nodes[n];
  if (x.kind == 0) { leaf_reach[x.leaf] = std::max(leaf_reach[x.leaf], reach); return; }
  double r = reach;
  for (int k : x.kids) {
    assign_reach(nodes, k, r, leaf_reach);
    if (x.kind == 1) r *= nodes[k].pass;
    else if (x.kind == 2) r *= 1.0 - nodes[k].pass;
  }
}

struct ThreadCtx {  // per calling thread: staging + events, created once
  PinnedBuf pinned;
  PinnedBuf readback;  // per-segment match counts + error word, copied back before the one stream sync
  PinnedBuf state_host;  // small dense states copied back with them (pg_execute)
  PinnedBuf ids_host;    // value-set ids of a finalize
  PinnedVec arena;              // pinned host image of the parameter arena (capacity reused across queries)
  std::vector<WorkItem> items;  // work items of the current query (capacity reused across queries)
  std::vector<WorkItem> items_perm;  // XCD-grouped order of the items (swapped with `items`)
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  // the overlapped list scan (stream plan's `split`): its first half runs on s2 beside the stream's second half
  hipStream_t s2 = nullptr;
  hipEvent_t ev_a = nullptr, ev_l = nullptr;
  int init() {
    if (ev[0]) return PG_OK;
    // timing-only events (phase times via hipEventElapsedTime; nothing waits on them for data): without the
    // system-scope fence a record costs no L2 write-back / invalidate between the dependent kernels it sits between
    for (auto& e : ev) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    HIP_CHECK(hipEventCreateWithFlags(&ev_a, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_l, hipEventDisableTiming));
    HIP_CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    return PG_OK;
  }
};
thread_local ThreadCtx t_ctx;

// A phase-timing event record (t_timing); PG_TIMING_EVENTS=0 skips them (dev A/B of their cost between kernels: the
// phase times then read 0)
hipError_t timing_record(hipEvent_t e, hipStream_t s) {
  static const bool off = getenv("PG_TIMING_EVENTS") && atoi(getenv("PG_TIMING_EVENTS")) == 0;
  return off ? hipSuccess : hipEventRecord(e, s);
}

bool pl_too_big(uint32_t ints) { return ints * 4ull > (uint64_t)kLdsSetBytes; }

// Upper bound of the scan grid: a whole number of resident rounds of blocks (2 x the resident blocks per CU, no
// partial last round).  Measured on config 2 / config 3: 6 -> 0.94 / 1.75 ms, 8 -> 0.97 / 1.93 ms, 5 -> 1.01 /
// 1.99 ms, 7 -> 1.03 / 2.01 ms.  `one_round`: one resident round (the XCD-grouped order).  PG_SCAN_BLOCKS_PER_CU
// overrides both.
uint64_t g_grid_caps[4] = {0, 0, 0, 0};
uint32_t g_num_cus = 256;
uint64_t g_wall_khz = 0;  // wall_clock64() ticks per ms (hipDeviceAttributeWallClockRate)
void init_grid_caps() {  // under g_init_mu (pg_init), before any query reads them
  int dev_cus = 0;
  if (hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, g_device) != hipSuccess || dev_cus <= 0)
    dev_cus = 256;
  g_num_cus = (uint32_t)dev_cus;
  int wall_khz = 0;
  if (hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, g_device) == hipSuccess && wall_khz > 0)
    g_wall_khz = (uint64_t)wall_khz;
  const char* e = getenv("PG_SCAN_BLOCKS_PER_CU");
  for (int i = 0; i < 4; i++) {
    const bool grouped = i & 1, one_round = i & 2;
    const int per_cu = e ? std::max(1, atoi(e)) : (one_round ? 1 : 2) * (int)scan_min_blocks_per_cu(grouped);
    g_grid_caps[i] = (uint64_t)dev_cus * per_cu;
  }
}
uint64_t scan_grid_cap(bool grouped, bool one_round = false) {
  return g_grid_caps[(grouped ? 1 : 0) + (one_round ? 2 : 0)];
}

int agg_layout(const pg_plan* plan, uint32_t integer, const std::vector<int32_t>& fx_shift,
               const std::vector<uint32_t>& fx_nwin, uint32_t special, std::vector<AggSpec>& aggs, uint32_t& n_i64,
               uint32_t& n_fx, uint32_t& n_min, uint32_t& n_max, uint32_t& bit_words) {
  n_i64 = 1;  // slot 0: doc count (COUNT, AVG count, group presence)
  n_fx = n_min = n_max = bit_words = 0;
  aggs.assign(plan->num_aggs, AggSpec{});
  for (uint32_t a = 0; a < plan->num_aggs; a++) {
    const pg_agg& g = plan->aggs[a];
    AggSpec& s2 = aggs[a];
    memset(&s2, 0, sizeof(s2));
    s2.fn = g.fn;
    s2.op = g.op;
    s2.sp_min = s2.sp_max = kNoSp;
    if (g.fn > PG_AGG_COUNTMV) return fail(PG_E_INVALID, "unknown aggregation %u", g.fn);
    if (g.op > PG_EXPR_SUB) return fail(PG_E_INVALID, "unknown expression op %u", g.op);
    if (g.flags & ~PG_AGG_MV_VALUES) return fail(PG_E_INVALID, "aggregation %u: unknown flags 0x%x", a, g.flags);
    s2.mv = (g.flags & PG_AGG_MV_VALUES) ? 1u : 0u;
    if (s2.mv && (g.fn == PG_AGG_COUNT || g.fn == PG_AGG_COUNTMV || g.op != PG_EXPR_COL))
      return fail(PG_E_INVALID, "aggregation %u: PG_AGG_MV_VALUES needs SUM / MIN / MAX / AVG / DISTINCTCOUNT of a column", a);
    switch (g.fn) {
      case PG_AGG_COUNT: s2.kind = SK_NONE; s2.slot = 0; break;
      case PG_AGG_COUNTMV: s2.kind = SK_I64; s2.slot = n_i64++; break;
      case PG_AGG_SUM: case PG_AGG_AVG:
        s2.integer = (integer >> a) & 1u;
        if (s2.integer) {
          s2.kind = SK_I64;
          s2.slot = n_i64++;
        } else {
          s2.kind = SK_FX;
          s2.slot = n_fx;
          s2.fx_shift = a < fx_shift.size() ? fx_shift[a] : fx_u0(-1074);
          s2.fx_nwin = a < fx_nwin.size() ? std::max(1u, std::min(fx_nwin[a], (uint32_t)kFxMaxWin)) : (uint32_t)kFxMaxWin;
          n_fx += s2.fx_nwin;
          if ((special >> a) & 1u) { s2.sp_min = n_min++; s2.sp_max = n_max++; }
        }
        s2.cnt_slot = (g.fn == PG_AGG_AVG && s2.mv) ? n_i64++ : 0;  // AVGMV counts values, not docs
        break;
      case PG_AGG_MIN: s2.kind = SK_MIN; s2.slot = n_min++; break;
      case PG_AGG_MAX: s2.kind = SK_MAX; s2.slot = n_max++; break;
      case PG_AGG_DISTINCTCOUNT:
        if (!g.key_cardinality) return fail(PG_E_INVALID, "DISTINCTCOUNT needs key_cardinality");
        s2.kind = SK_BITS;
        s2.key_kind = g.key_kind;
        s2.key_card = g.key_cardinality;
        s2.key_base = g.key_base;
        s2.dc_word = bit_words;
        bit_words += (g.key_cardinality + 31) / 32;
        break;
    }
  }
  return PG_OK;
}

int Partials::alloc_state(hipStream_t s, bool init, FillSpans* defer) {
  const uint64_t G = num_slots;
  int rc;
  const bool hash = mode == GM_HASH || mode == GM_HASH_SEG;
  if ((rc = i64.alloc_pooled(G * 8ull * n_i64))) return rc;
  if (n_fx) { if ((rc = fx.alloc_pooled(G * 16ull * n_fx))) return rc; } else fx.reset();
  if (n_min) { if ((rc = mn.alloc_pooled(G * 8ull * n_min))) return rc; } else mn.reset();
  if (n_max) { if ((rc = mx.alloc_pooled(G * 8ull * n_max))) return rc; } else mx.reset();
  if (bit_words) { if ((rc = bits.alloc_pooled(G * 4ull * bit_words))) return rc; } else bits.reset();
  if (hash) { if ((rc = keys.alloc_pooled(G * 8ull))) return rc; } else keys.reset();
  if (mode == GM_HASH_SEG) { if ((rc = first_doc.alloc_pooled(G * 8ull))) return rc; } else first_doc.reset();
  if ((rc = misc.alloc_pooled(16))) return rc;
  if (init) HIP_CHECK(launch_init_view(view(), s, defer));
  else HIP_CHECK(hipMemsetAsync(misc.p, 0, 16, s));  // every slot is written by the producer (pg_part.hip)
  return PG_OK;
}

// A dense state of at most this many bytes is finalised on the host from one D2H copy (config 2: 90 x 3 int64):
// the device path's select / final-value / trim launches and its two stream round trips cost ~0.1 ms there.  Under
// pg_execute (no cross-GPU merge in between) the copy is queued right behind the scan, before its one sync.
constexpr uint64_t kHostFinalBytes = 1ull << 20;
thread_local bool t_prefetch_state = false;  // set by pg_execute around its pg_execute_partial

constexpr int kRetryLargerTable = 1;  // internal: the hash table overflowed its fill budget
constexpr int kRetryNoStream = 2;     // internal: a selective-stream region overflowed (more survivors than estimated)
constexpr int kRetryExactPart = 3;    // internal: a speculative GM_PART region overflowed (skewed keys): exact offsets

// Pooled device scratch of a host-side sequence of small launches (freed after the caller synchronises).
struct Scratch {
  hipStream_t s;
  std::vector<DevBuf> bufs;
  explicit Scratch(hipStream_t st) : s(st) {}
  ~Scratch() { if (!bufs.empty()) (void)hipStreamSynchronize(s); }  // before the blocks return to the pool
  template <class T> T* get(uint64_t n, int& rc) {
    bufs.emplace_back();
    rc = bufs.back().alloc_pooled(n * sizeof(T) + 16);
    return rc ? nullptr : (T*)bufs.back().p;
  }
};

// OR of the order keys and OR of their complements (order_keys_kernel's span)
struct KeySpan {
  uint64_t any, anyz;
};

// Copy one device value to the host (synchronous on s).
template <class T> int read_back(const T* d, T& h, hipStream_t s) {
  HIP_CHECK(hipMemcpyAsync(&h, d, sizeof(T), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return PG_OK;
}

// A fresh GM_HASH state with the layout of `src` and room for `groups` groups.
int hash_like(const Partials& src, uint64_t groups, Partials& out, hipStream_t s) {
  out.mode = GM_HASH;
  out.num_slots = pow2_at_least(std::max<uint64_t>(1024, 2 * groups));
  const uint64_t slot_bytes = 8ull * (src.n_i64 + 2ull * src.n_fx + src.n_min + src.n_max) + 4ull * src.bit_words + 12;
  if (out.num_slots > kMaxHashSlots || out.num_slots * slot_bytes > kStateBudget)  // compile_and_run's budget
    return fail(PG_E_UNSUPPORTED, "merge table of %llu groups (%llu slots x %llu bytes) exceeds the state budget",
                (unsigned long long)groups, (unsigned long long)out.num_slots, (unsigned long long)slot_bytes);
  out.max_fill = (uint32_t)(out.num_slots / 4 * 3);
  out.n_i64 = src.n_i64; out.n_fx = src.n_fx; out.n_min = src.n_min; out.n_max = src.n_max;
  out.bit_words = src.bit_words;
  out.key_card = src.key_card;
  out.key_stride = src.key_stride;
  out.projected_cols = src.projected_cols;
  out.total_docs = src.total_docs;
  out.num_segments = src.num_segments;
  out.layout = src.layout;
  out.flags = src.flags;
  out.aggs = src.aggs;
  return out.alloc_state(s);
}

// numGroupsLimit (IntGroupIdMap.getGroupId, DictionaryBasedGroupKeyGenerator.java:991-1016): every segment of a
// GM_HASH_SEG table keeps the `limit` keys seen first (its group ids 0..limit-1; docs of later keys got INVALID_ID and
// were dropped) -- first matching doc, then (mv: multi-value keys) the key's position among that doc's key tuples in
// getIntRawKeys order (:472-540); the kept (segment, key) states are then merged by key (GroupByOrderByCombineOperator)
// into a GM_HASH table that replaces P's state.
int truncate_and_merge(Partials& P, uint64_t limit, bool mv, hipStream_t s) {
  const StateView v = P.view();
  const uint64_t cap = P.num_slots;
  Scratch sc(s);
  int rc = PG_OK;
  const size_t temp_bytes = std::max(select_temp_bytes(cap), sort_temp_bytes(cap));
  uint32_t* slots = sc.get<uint32_t>(cap, rc);
  uint32_t* d_num = sc.get<uint32_t>(2, rc);
  void* temp = sc.get<uint8_t>(temp_bytes, rc);
  if (rc) return rc;
  HIP_CHECK(launch_select_slots(v, SEL_OCCUPIED, 0, 1, slots, d_num, temp, temp_bytes, s));
  uint32_t n = 0;
  if ((rc = read_back(d_num, n, s))) return rc;
  uint64_t* tmp_keys = sc.get<uint64_t>(n + 1, rc);
  uint64_t* sorted_keys = sc.get<uint64_t>(n + 1, rc);
  uint32_t* sorted_slots = sc.get<uint32_t>(n + 1, rc);
  uint32_t* seg_first = sc.get<uint32_t>(P.num_segments + 1, rc);
  uint8_t* keep = sc.get<uint8_t>(n + 1, rc);
  uint32_t* kept = sc.get<uint32_t>(n + 1, rc);
  unsigned int* reached = sc.get<unsigned int>(1, rc);
  if (rc) return rc;
  HIP_CHECK(hipMemsetAsync(reached, 0, 4, s));
  HIP_CHECK(launch_seg_truncate(v, slots, n, P.num_segments, limit, mv, tmp_keys, sorted_keys, sorted_slots, seg_first,
                                keep, reached, temp, temp_bytes, s));
  uint32_t hit = 0;
  if ((rc = read_back((uint32_t*)reached, hit, s))) return rc;
  if (hit) P.flags |= PG_RESULT_GROUPS_LIMIT_REACHED;
  uint32_t nk = 0;
  if (n) {
    HIP_CHECK(launch_select_flagged(sorted_slots, keep, n, kept, d_num, temp, temp_bytes, s));
    if ((rc = read_back(d_num, nk, s))) return rc;
  }
  const uint64_t rb = row_bytes(v);
  uint8_t* rows = sc.get<uint8_t>(rb * (nk + 1), rc);
  if (rc) return rc;
  HIP_CHECK(launch_gather_rows(v, kept, nk, P.num_segments, rows, s));
  Partials H;
  if ((rc = hash_like(P, nk, H, s))) return rc;
  HIP_CHECK(launch_merge_rows(H.view(), rows, nk, s));
  uint32_t fe[2] = {0, 0};
  HIP_CHECK(hipMemcpyAsync(fe, H.misc.p, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (fe[1]) return fail(PG_E_INVALID, "truncation merge overflowed its table (code %u)", fe[1]);
  P.mode = GM_HASH;
  P.num_slots = H.num_slots;
  P.max_fill = H.max_fill;
  P.keys = std::move(H.keys);
  P.i64 = std::move(H.i64);
  P.fx = std::move(H.fx);
  P.mn = std::move(H.mn);
  P.mx = std::move(H.mx);
  P.bits = std::move(H.bits);
  P.misc = std::move(H.misc);
  P.first_doc.reset();
  return PG_OK;
}

// The segment's filter is match-all after FilterPlanNode's pruning (FilterOperatorUtils: AND drops match-all children,
// OR with a match-all child is match-all, NOT(empty) is match-all): three-valued evaluation of the postfix program.
// A leaf's dictIds sorted, unique and in [0, card) (they index LUTs on the device).  Branch-free so it vectorises
// (IN lists of 1 000 ids x 128 segments cost 85 us per query with a branch per id); an AVX2 build of the same loop
// when the host has it (8 lanes instead of SSE2's 4).
template <int V>
static inline uint32_t ids_bad(const int32_t* ids, uint32_t n, uint32_t card) {
  uint32_t bad = n ? (uint32_t)((uint32_t)ids[0] >= card) : 0u;  // negative ids are >= card as uint32
  for (uint32_t i = 1; i < n; i++) bad |= (uint32_t)(ids[i] <= ids[i - 1]) | (uint32_t)((uint32_t)ids[i] >= card);
  return bad;
}
__attribute__((target("avx2"))) static uint32_t ids_bad_avx2(const int32_t* ids, uint32_t n, uint32_t card) {
  return ids_bad<2>(ids, n, card);
}
bool ids_valid(const int32_t* ids, uint32_t n, uint32_t card) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  return (avx2 ? ids_bad_avx2(ids, n, card) : ids_bad<1>(ids, n, card)) == 0;
}

bool filter_is_match_all(const pg_plan* plan, const pg_leaf* leaves) {
  if (!plan->num_ops) return true;
  std::vector<int> st;
  for (uint32_t i = 0; i < plan->num_ops; i++) {
    const int32_t op = plan->ops[i];
    if (op >= 0) {
      st.push_back(leaves[op].kind == PG_LEAF_MATCH_ALL ? 1 : leaves[op].kind == PG_LEAF_EMPTY ? 0 : -1);
    } else if (op == PG_OP_NOT) {
      st.back() = st.back() < 0 ? -1 : !st.back();
    } else {
      const int n = (-op) & 0xFF;
      const bool is_and = ((-op) & 0x300) == 0x100;
      int v = is_and ? 1 : 0;
      for (int k = 0; k < n; k++) {
        const int x = st[st.size() - 1 - k];
        if (is_and) v = (v == 0 || x == 0) ? 0 : (v < 0 || x < 0 ? -1 : 1);
        else v = (v == 1 || x == 1) ? 1 : (v < 0 || x < 0 ? -1 : 0);
      }
      st.resize(st.size() - n);
      st.push_back(v);
    }
  }
  return st.size() == 1 && st[0] == 1;
}

// Aggregation inputs that only need dictionary VALUES (not dictIds) may read a column's decoded forward index.
bool agg_decodes(const pg_agg& g) {
  if (g.flags & PG_AGG_MV_VALUES) return false;  // MV values: dictIds through the row offsets + dictionary
  return g.fn == PG_AGG_SUM || g.fn == PG_AGG_MIN || g.fn == PG_AGG_MAX || g.fn == PG_AGG_AVG ||
         (g.fn == PG_AGG_DISTINCTCOUNT && g.key_kind == PG_KEY_VALUE_OFFSET);
}
void use_decoded(ColDesc& dc, const ColumnRes* c) {
  const DevBuf& w = c->identity ? c->words : c->vals;
  dc.words = (const uint32_t*)w.p;
  dc.wbytes = (uint32_t)std::min<uint64_t>(w.bytes, 0xFFFFFFF0ull);
  dc.bits = c->identity ? c->bits : c->vbits;
  dc.dict = nullptr;
  dc.card = 0xFFFFFFFFu;
  dc.vbase = c->imin;
  dc.decoded = 1;
  dc.identity = c->identity ? 1u : 0u;
}

// The scan's descriptor of group key column `c` (dictIds + dictionary / keymap, or the decoded forward index when the
// key is a value offset of a column that has one).
void key_coldesc(ColDesc& dc, const ColumnRes* c, const pg_key& key) {
  memset(&dc, 0, sizeof(dc));
  if (c->fwd == FWD_RAW) {  // a raw INT / LONG key (value offsets): the range index's packed offsets, else the values
    dc.dtype = c->dtype;
    if (c->vals.p) {
      use_decoded(dc, c);
    } else {  // "dictId" = doc id (bits 0), "dictionary" = the values, as for a raw aggregation input
      dc.dict = c->rawv.p;
      dc.card = c->num_docs;
    }
    return;
  }
  dc.words = (const uint32_t*)c->words.p;
  dc.wbytes = (uint32_t)std::min<uint64_t>(c->words.bytes, 0xFFFFFFF0ull);
  dc.dict = c->dict.p;
  dc.keymap = (const int32_t*)c->keymap.p;
  dc.mv_offsets = (const uint32_t*)c->mv_offsets.p;  // MV: the doc's values are words [off[d], off[d + 1])
  dc.bits = c->bits;
  dc.dtype = c->dtype;
  dc.card = c->card;
  if (c->fwd != FWD_MV && key.kind == PG_KEY_VALUE_OFFSET && (c->vals.p || c->identity)) use_decoded(dc, c);
}

// A group key column usable in segment si: SV dictIds + dictionary (any key kind), or a raw INT / LONG forward index
// as value offsets (NoDictionarySingleColumnGroupKeyGenerator.java:51 / NoDictionaryMultiColumnGroupKeyGenerator.java:49
// key raw values; here the value offset is the key id, so segments and GPUs merge by value as for dictionary keys).
// A multi-value dictionary column (allow_mv: one of the plan's MV keys) groups each of a doc's values
// (DictionaryBasedGroupKeyGenerator.generateKeysForBlock(.., int[][]) :188-200).
int check_key_column(const ColumnRes* c, const pg_key& key, uint32_t k, uint32_t si, bool allow_mv = false) {
  if (!c) return fail(PG_E_NOTFOUND, "group key column %u not resident in segment %u", key.col_id, si);
  const bool raw = c->fwd == FWD_RAW;
  if ((!c->has_dict && !raw) || c->fwd == FWD_NONE || (c->fwd == FWD_MV && (!allow_mv || !c->mv_offsets.p)))
    return fail(PG_E_UNSUPPORTED, "group key column %u unusable in segment %u", key.col_id, si);
  if (raw && (key.kind != PG_KEY_VALUE_OFFSET || c->dtype > PG_LONG))
    return fail(PG_E_UNSUPPORTED, "raw group key column %u: value-offset INT / LONG keys only", key.col_id);
  if (c->dtype > PG_DOUBLE && key.kind != PG_KEY_KEYMAP)
    return fail(PG_E_INVALID, "non-numeric key column %u needs a keymap", key.col_id);
  if (key.kind == PG_KEY_KEYMAP && !c->has_keymap) return fail(PG_E_NOTFOUND, "keymap missing for column %u", key.col_id);
  if (key.kind == PG_KEY_VALUE_OFFSET && c->dtype != PG_INT && c->dtype != PG_LONG)
    return fail(PG_E_INVALID, "VALUE_OFFSET key on non-integer column %u", key.col_id);
  const bool has_values = raw ? c->num_docs > 0 : c->card > 0;
  if (key.kind == PG_KEY_VALUE_OFFSET && has_values &&
      (c->imin < key.base || (uint64_t)(c->imax - key.base) >= key.cardinality))
    return fail(PG_E_INVALID, "column %u values outside the key range of key %u", key.col_id, k);
  return PG_OK;
}

// Wide group keys (pg_wide.hip): the plan is run with one key, the doc's tuple slot, read from a per-segment column
// that exists only for this query; compile_and_run's column lookup finds it under kWideColId.
constexpr uint32_t kWideColId = 0xFFFFFFF0u;
thread_local const std::vector<ColumnRes>* t_wide_cols = nullptr;

// The physical form a compiled leaf took (pinot_trace.h pg_leaf_form).
uint32_t leaf_form(const pg_leaf& pl, const LeafDesc& dl) {
  if (dl.kind == LK_ALL) return PG_FORM_MATCH_ALL;
  if (dl.kind == LK_NONE) return PG_FORM_EMPTY;
  switch (pl.kind) {
    case PG_LEAF_SV_SCAN:
      return dl.kind == LK_SET_LDS ? PG_FORM_SCAN_SET_LDS : dl.kind == LK_SET_LUT ? PG_FORM_SCAN_SET_LUT : PG_FORM_SCAN_RANGE;
    case PG_LEAF_SORTED: return dl.kind == LK_DOCRANGE ? PG_FORM_SORTED_RANGE : PG_FORM_SORTED_BITMAP;
    case PG_LEAF_INVERTED: return PG_FORM_INVERTED;
    case PG_LEAF_MV_SCAN: return PG_FORM_MV_SCAN;
    case PG_LEAF_RAW_SCAN: return PG_FORM_RAW_SCAN;
    case PG_LEAF_RANGE_INDEX: return PG_FORM_RANGE_INDEX;
    default: return PG_FORM_EMPTY;
  }
}

// ---- SUM / AVG accumulation layout from the columns' value bounds (compile_and_run, and the multi-device layout that
// makes every logical device's partial state agree, global_layout)
struct SumBounds {
  double bound_a = 0, bound_b = 0, fin_a = 0, fin_b = 0;  // |value| bounds: all values / the finite ones
  double low_a = 0, low_b = 0;                            // smallest nonzero finite |value| (0 = none)
  bool all_int = true, nonfinite = false;
};
inline double low_min(double x, double y) { return x == 0 ? y : (y == 0 ? x : std::min(x, y)); }
void sum_bounds_add(SumBounds& b, const ColumnRes* ca, const ColumnRes* cb) {
  b.all_int &= ca->dtype <= PG_LONG;
  b.bound_a = std::max(b.bound_a, std::max(fabs(ca->dmin), fabs(ca->dmax)));
  b.fin_a = std::max(b.fin_a, ca->fin_abs);
  b.low_a = low_min(b.low_a, ca->fin_min);
  b.nonfinite |= ca->nonfinite;
  if (cb) {
    b.all_int &= cb->dtype <= PG_LONG;
    b.bound_b = std::max(b.bound_b, std::max(fabs(cb->dmin), fabs(cb->dmax)));
    b.fin_b = std::max(b.fin_b, cb->fin_abs);
    b.low_b = low_min(b.low_b, cb->fin_min);
    b.nonfinite |= cb->nonfinite;
  }
}
// integer-exact accumulation when every partial sum provably fits in int64 (2^62 margin); identical to the reference's
// double accumulation while |sum| < 2^53, more exact beyond (within the 1e-9 tolerance)
bool sum_as_int(const SumBounds& b, const pg_agg& g, bool two, uint32_t plan_flags, uint64_t docs) {
  double vb = b.bound_a;
  if (two) vb = g.op == PG_EXPR_MUL ? b.bound_a * b.bound_b : b.bound_a + b.bound_b;
  return b.all_int && !(plan_flags & PG_PLAN_F64_SUMS) && vb * (double)(docs ? docs : 1) < 4.0e18;
}
// SK_FX: exponent windows from power-of-two bounds 2^klo <= |x| <= 2^khi of the nonzero finite inputs (an expression of
// finite operands can still overflow to +-inf: then the upper bound is DBL_MAX's and the non-finite results go to the
// special slots; a product can underflow: its lower bound is the smallest subnormal).  a*b: the products of the bounds;
// a+b / a-b: the larger bound doubled, and a nonzero result is a multiple of the smaller operand's last mantissa bit
// (2^-52 of its lower bound).  `any`: some input may be nonzero.
void sum_windows(const SumBounds& b, const pg_agg& g, bool two, int& klo, int& khi, bool& nonfinite, bool& any) {
  double fb = b.fin_a, lb = b.low_a;
  nonfinite = b.nonfinite;
  if (two) {
    if (g.op == PG_EXPR_MUL) {
      fb = b.fin_a * b.fin_b;
      lb = b.low_a * b.low_b;
      if (b.low_a > 0 && b.low_b > 0 && lb == 0) lb = 4.9406564584124654e-324;
    } else {
      fb = b.fin_a + b.fin_b;
      lb = ldexp(low_min(b.low_a, b.low_b), -52);
      if (low_min(b.low_a, b.low_b) > 0 && lb == 0) lb = 4.9406564584124654e-324;
    }
  }
  if (!std::isfinite(fb)) { fb = DBL_MAX; nonfinite = true; }
  khi = klo = 0;
  if (fb > 0) (void)frexp(fb, &khi);  // fb < 2^khi
  if (lb > 0) { (void)frexp(lb, &klo); klo -= 1; }  // lb >= 2^klo
  else klo = khi;
  any = fb > 0;
}

// Multi-device layout hint (execute_partial_multi -> each logical device's compile_and_run): the layout choices that
// must agree between the partial states being merged, decided once over the whole plan.
struct LayoutHint {
  bool on = false;
  uint64_t docs = 0;       // the whole plan's docs (dense-vs-hash sizing)
  uint32_t integer = 0;    // bit a: SUM / AVG a accumulates integer-exact
};
thread_local LayoutHint t_layout;

int compile_and_run(const pg_plan* plan, Partials& P, pg_stats& stats, uint64_t hash_cap, bool allow_stream,
                    bool allow_spec) {
  const double t_enter = wall_ms();
  if (!plan) return fail(PG_E_INVALID, "null plan");
  // this attempt's recording (a rerun starts over; the wide-key path's first pass is kept)
  memset(t_trace.leaf_forms, 0, sizeof(t_trace.leaf_forms));
  t_trace.path &= PG_PATH_WIDE_KEYS;
  t_trace.num_leaves = plan->num_leaves;
  t_trace.num_segments = plan->num_segments;
  if (plan->abi_version != PG_ABI_VERSION) return fail(PG_E_INVALID, "ABI version %u != %u", plan->abi_version, PG_ABI_VERSION);
  if (plan->num_aggs > (uint32_t)kMaxAggs) return fail(PG_E_UNSUPPORTED, "more than %d aggregations", kMaxAggs);
  if (plan->num_keys > (uint32_t)kMaxKeys) return fail(PG_E_UNSUPPORTED, "more than %d group-by keys", kMaxKeys);
  if (plan->num_leaves > (uint32_t)kMaxLeaves) return fail(PG_E_UNSUPPORTED, "more than %d filter leaves", kMaxLeaves);
  if (plan->num_segments && !plan->segments) return fail(PG_E_INVALID, "null segment list");
  if ((plan->num_aggs && !plan->aggs) || (plan->num_keys && !plan->keys) || (plan->num_ops && !plan->ops))
    return fail(PG_E_INVALID, "null aggregation / key / filter array");
  // validate the postfix program
  {
    int sp = 0, mx = 0;
    for (uint32_t i = 0; i < plan->num_ops; i++) {
      const int32_t op = plan->ops[i];
      if (op >= 0) {
        if ((uint32_t)op >= plan->num_leaves) return fail(PG_E_INVALID, "op %u references leaf %d", i, op);
        sp++;
      } else if (op == PG_OP_NOT) {
        if (sp < 1) return fail(PG_E_INVALID, "NOT on empty stack");
      } else {
        const int n = (-op) & 0xFF;
        if (n < 1 || sp < n || !((-op) & 0x300) || ((-op) & ~0x3FF)) return fail(PG_E_INVALID, "bad AND/OR at op %u", i);
        sp -= n - 1;
      }
      mx = std::max(mx, sp);
    }
    if (plan->num_ops && sp != 1) return fail(PG_E_INVALID, "filter program leaves %d values", sp);
    if (mx > 64) return fail(PG_E_UNSUPPORTED, "filter program too deep");
  }
  if (plan->deadline_ms && now_ms() > plan->deadline_ms) return fail(PG_E_TIMEOUT, "deadline passed before launch");
  if (is_cancelled(plan->query_id)) return fail(PG_E_CANCELLED, "query %llu cancelled", (unsigned long long)plan->query_id);
  int rc = t_ctx.init();
  if (rc) return rc;

  hipStream_t s = plan->stream ? (hipStream_t)plan->stream : thread_stream();
  std::shared_lock<std::shared_mutex> lk(g_seg_mu);

  const uint32_t S = plan->num_segments, L = plan->num_leaves, A = plan->num_aggs, K = plan->num_keys;
  std::vector<const SegmentRes*> segs(S);
  auto col = [&](uint32_t si, uint32_t cid) -> const ColumnRes* {
    if (cid == kWideColId && t_wide_cols) return &(*t_wide_cols)[si];
    auto it = segs[si]->cols.find(cid);
    return it == segs[si]->cols.end() ? nullptr : &it->second;
  };
  for (uint32_t si = 0; si < S; si++) {
    auto it = g_segs.find(plan->segments[si].seg_key);
    if (it == g_segs.end()) return fail(PG_E_NOTFOUND, "segment %llu not resident", (unsigned long long)plan->segments[si].seg_key);
    segs[si] = it->second;
    if (it->second->ldev != (uint32_t)t_ldev)
      return fail(PG_E_STATE, "segment %llu is resident on logical device %u, not %d",
                  (unsigned long long)plan->segments[si].seg_key, it->second->ldev, t_ldev);
    if (L && !plan->segments[si].leaves) return fail(PG_E_INVALID, "segment %u has no leaves", si);
  }

  PG_PROF("lower_cols");
  // ---- RangeIndexBasedFilterOperator leaves (PG_LEAF_RANGE_INDEX): lowered onto the forms that evaluate them.  A
  // dictionary column's range index answers dictIds [lo, hi) -> the packed forward index (SV scan form); a raw INT /
  // LONG column's becomes a dictId-like range over its packed (value - min) offsets (kind kept RANGE_INDEX, its own
  // staging slot); a raw FLOAT / DOUBLE column's is the raw compare.  All are exact index leaves: no entries
  // scanned in the filter (BitSlicedRangeIndexReader.isExact, RangeIndexBasedFilterOperator.java:62-67).
  pg_plan shadow;
  std::vector<pg_segment_ref> shadow_segs;
  std::vector<pg_leaf> shadow_leaves;
  std::vector<uint8_t> index_leaf((uint64_t)S * L, 0);
  {
    bool any = false;
    for (uint32_t si = 0; si < S && !any; si++)
      for (uint32_t li = 0; li < L; li++) any |= plan->segments[si].leaves[li].kind == PG_LEAF_RANGE_INDEX;
    if (any) {
      shadow = *plan;
      shadow_segs.assign(plan->segments, plan->segments + S);
      shadow_leaves.resize((uint64_t)S * L);
      for (uint32_t si = 0; si < S; si++) {
        std::copy(plan->segments[si].leaves, plan->segments[si].leaves + L, &shadow_leaves[(uint64_t)si * L]);
        shadow_segs[si].leaves = &shadow_leaves[(uint64_t)si * L];
        for (uint32_t li = 0; li < L; li++) {
          pg_leaf& pl = shadow_leaves[(uint64_t)si * L + li];
          if (pl.kind != PG_LEAF_RANGE_INDEX) continue;
          const ColumnRes* c = col(si, pl.col_id);
          if (!c) return fail(PG_E_NOTFOUND, "leaf %u: column %u not resident in segment %u", li, pl.col_id, si);
          if (!c->has_range) return fail(PG_E_INVALID, "range-index leaf on column %u without a range index", pl.col_id);
          if (pl.num_ids) return fail(PG_E_INVALID, "range-index leaf %u with a value list (RANGE predicates only)", li);
          index_leaf[(uint64_t)si * L + li] = 1;
          if (c->fwd != FWD_RAW) { pl.kind = PG_LEAF_SV_SCAN; continue; }
          if (!c->vals.p) { pl.kind = PG_LEAF_RAW_SCAN; continue; }
          // closed [ilo, ihi] on the values -> [lo, hi) on the offsets (value - imin); vbits <= 30 keeps both in int32
          const int64_t lo = std::max(pl.ilo, c->imin), hi = std::min(pl.ihi, c->imax);
          pl.lo = lo > hi ? 0 : (int32_t)(lo - c->imin);
          pl.hi = lo > hi ? 0 : (int32_t)(hi - c->imin + 1);
        }
      }
      shadow.segments = shadow_segs.data();
      plan = &shadow;
    }
  }

  QuerySpec q;
  memset(&q, 0, sizeof(q));
  q.num_segments = S;
  q.num_leaves = L;
  q.num_aggs = A;
  q.num_keys = K;

  PG_PROF("keys");
  // ---- group key space: packed key = mixed radix of the table-global key ids, first key least significant
  // (DictionaryBasedGroupKeyGenerator raw keys, :280-322, over table-global ids so segments merge by value)
  uint64_t G = 1;
  bool g_over = false;
  P.key_card.assign(K, 0);
  P.key_stride.assign(K, 0);
  for (uint32_t k = 0; k < K; k++) {
    const pg_key& key = plan->keys[k];
    if (key.cardinality == 0) return fail(PG_E_INVALID, "group key %u has zero cardinality", k);
    if (key.kind > PG_KEY_KEYMAP) return fail(PG_E_INVALID, "group key %u: unknown kind %u", k, key.kind);
    q.key_kind[k] = key.kind;
    q.key_card[k] = key.cardinality;
    q.key_base[k] = key.base;
    q.key_stride[k] = G;
    P.key_card[k] = key.cardinality;
    P.key_stride[k] = G;
    if (G > (~0ull) / key.cardinality) g_over = true;
    else G *= key.cardinality;
  }
  if (K && (g_over || G >= (1ull << 62)))
    return fail(PG_E_UNSUPPORTED, "packed group key of %u keys exceeds 62 bits", K);
  // numGroupsLimit: a segment keeps the first `limit` distinct keys in doc order (IntGroupIdMap :991-1016).  It can
  // only bite in a segment whose matching docs or key-cardinality product exceed the limit (the array-based holder,
  // card product <= maxInitialResultHolderCapacity <= limit, never truncates).
  const uint64_t limit = plan->num_groups_limit ? plan->num_groups_limit : kDefaultNumGroupsLimit;
  uint64_t seg_groups = 0;  // sum over segments of an upper bound of the segment's distinct keys
  bool truncating = false;
  q.mv_keys = 0;
  if (K) {
    // the multi-value keys: a doc joins the group of every tuple of the cartesian product of their lists
    // (DictionaryBasedGroupKeyGenerator.getIntRawKeys :472-540)
    {
      for (uint32_t k = 0; k < K && S; k++) {
        bool mv = false;
        for (uint32_t si = 0; si < S; si++) {
          const ColumnRes* c = col(si, plan->keys[k].col_id);
          mv |= c && c->fwd == FWD_MV;
        }
        if (mv) q.mv_keys |= 1u << k;
      }
    }
    for (uint32_t si = 0; si < S; si++) {
      uint64_t prod = 1;
      for (uint32_t k = 0; k < K; k++) {
        const ColumnRes* c = col(si, plan->keys[k].col_id);
        if ((rc = check_key_column(c, plan->keys[k], k, si, (q.mv_keys >> k) & 1u))) return rc;
        if (((q.mv_keys >> k) & 1u) && c->fwd != FWD_MV)
          return fail(PG_E_UNSUPPORTED, "group key %u is multi-value in some segments only", k);
        // distinct values in the segment: the dictionary's size, or (raw) at most its docs and the key range
        const uint64_t kc = c->fwd == FWD_RAW ? std::min<uint64_t>(c->num_docs, plan->keys[k].cardinality) : c->card;
        prod = prod > (1ull << 62) / (kc ? kc : 1) ? (1ull << 62) : prod * kc;
      }
      // (an MV key: a doc may hold several groups -- bounded by the key space, not the docs)
      const uint64_t ub = q.mv_keys ? prod : std::min<uint64_t>(prod, plan->segments[si].num_docs);
      seg_groups += ub;
      // >=: a segment holding exactly `limit` keys reports numGroupsLimitReached (getNumGroups() >= limit,
      // AggregationGroupByOrderByOperator.java:112-113), which the per-segment table counts
      truncating |= ub >= limit;
    }
  }

  PG_PROF("aggs");
  // ---- aggregation state layout
  uint64_t total_docs = 0;
  for (uint32_t si = 0; si < S; si++) total_docs += plan->segments[si].num_docs;
  std::unordered_set<uint32_t> projected;
  uint32_t integer = 0, special = 0;
  std::vector<int32_t> fx_shift(A, 0);
  std::vector<uint32_t> fx_nwin(A, 1);
  for (uint32_t a = 0; a < A; a++) {
    const pg_agg& g = plan->aggs[a];
    if (g.fn > PG_AGG_COUNTMV) return fail(PG_E_INVALID, "unknown aggregation %u", g.fn);
    if (g.op > PG_EXPR_SUB) return fail(PG_E_INVALID, "unknown expression op %u", g.op);
    if (g.fn == PG_AGG_COUNT) continue;
    projected.insert(g.col_a & ~PG_COL_DERIVED);
    const bool two = (g.fn == PG_AGG_SUM || g.fn == PG_AGG_MIN || g.fn == PG_AGG_MAX || g.fn == PG_AGG_AVG) && g.op != PG_EXPR_COL;
    if (two) projected.insert(g.col_b & ~PG_COL_DERIVED);
    SumBounds sb;
    const bool mv = (g.flags & PG_AGG_MV_VALUES) != 0;
    uint64_t mv_vals = 0;  // MV values: the inputs the integer-exactness bound counts (not the docs)
    if (mv) q.mv_aggs |= 1u << a;
    for (uint32_t si = 0; si < S; si++) {
      const ColumnRes* ca = col(si, g.col_a);
      if (!ca) return fail(PG_E_NOTFOUND, "aggregation %u: column %u not resident in segment %u", a, g.col_a, si);
      if (g.fn == PG_AGG_COUNTMV) {
        if (ca->fwd != FWD_MV) return fail(PG_E_INVALID, "COUNTMV on a single-value column %u", g.col_a);
        continue;
      }
      const bool raw_a = ca->fwd == FWD_RAW;
      if (mv != (ca->fwd == FWD_MV))
        return fail(PG_E_UNSUPPORTED, "aggregation %u: column %u is %s-value", a, g.col_a, mv ? "single" : "multi");
      if (mv && (!ca->mv_offsets.p || !ca->has_dict))
        return fail(PG_E_UNSUPPORTED, "aggregation %u: MV column %u needs its row offsets + dictionary", a, g.col_a);
      mv_vals += ca->num_values;
      if (ca->fwd == FWD_NONE || (!ca->has_dict && !raw_a))
        return fail(PG_E_UNSUPPORTED, "aggregation %u: column %u needs an SV forward index + dictionary", a, g.col_a);
      if (raw_a && g.fn == PG_AGG_DISTINCTCOUNT && g.key_kind != PG_KEY_VALUE_OFFSET)
        return fail(PG_E_UNSUPPORTED, "DISTINCTCOUNT of raw column %u needs value-offset ids", g.col_a);
      if (g.fn == PG_AGG_DISTINCTCOUNT) {
        if (g.key_kind == PG_KEY_KEYMAP && !ca->has_keymap) return fail(PG_E_NOTFOUND, "DISTINCTCOUNT keymap missing");
        if (g.key_kind != PG_KEY_KEYMAP && g.key_kind != PG_KEY_VALUE_OFFSET) return fail(PG_E_INVALID, "bad key kind");
        if (g.key_kind == PG_KEY_VALUE_OFFSET && ca->card &&
            (ca->dtype > PG_LONG || ca->imin < g.key_base || (uint64_t)(ca->imax - g.key_base) >= g.key_cardinality))
          return fail(PG_E_INVALID, "DISTINCTCOUNT values outside the key range");
        continue;
      }
      if (ca->dtype > PG_DOUBLE) return fail(PG_E_UNSUPPORTED, "numeric aggregation on non-numeric column %u", g.col_a);
      const ColumnRes* cb = nullptr;
      if (two) {
        cb = col(si, g.col_b);
        if (!cb || cb->fwd == FWD_NONE || cb->fwd == FWD_MV || (!cb->has_dict && cb->fwd != FWD_RAW) || cb->dtype > PG_DOUBLE)
          return fail(PG_E_UNSUPPORTED, "aggregation %u: second operand column %u unusable", a, g.col_b);
      }
      sum_bounds_add(sb, ca, cb);
    }
    if (g.fn == PG_AGG_SUM || g.fn == PG_AGG_AVG) {
      const bool as_int = t_layout.on ? ((t_layout.integer >> a) & 1u) != 0
                                      : sum_as_int(sb, g, two, plan->flags, mv ? mv_vals : total_docs);
      if (as_int) {
        integer |= 1u << a;
      } else {
        int klo, khi;
        bool nonfinite, any;
        sum_windows(sb, g, two, klo, khi, nonfinite, any);
        if (g.sum_flags & PG_SUM_BOUNDS) {  // the caller's table-global bounds (the same windows on every GPU / server)
          if (any && (khi > g.sum_exp || klo < g.sum_exp_lo))
            return fail(PG_E_INVALID, "aggregation %u: inputs in [2^%d, 2^%d] exceed the plan's sum bounds [2^%d, 2^%d]",
                        a, klo, khi, g.sum_exp_lo, g.sum_exp);
          khi = g.sum_exp;
          klo = g.sum_exp_lo;
        }
        if (klo < -1100 || khi > 1024 || klo > khi)
          return fail(PG_E_INVALID, "aggregation %u: sum bounds [2^%d, 2^%d] out of range", a, klo, khi);
        fx_shift[a] = fx_u0(klo);
        fx_nwin[a] = fx_num_windows(klo, khi);
        if (nonfinite || (g.sum_flags & PG_SUM_NONFINITE)) special |= 1u << a;
      }
    }
  }
  {
    int rc2 = agg_layout(plan, integer, fx_shift, fx_nwin, special, P.aggs, P.n_i64, P.n_fx, P.n_min, P.n_max, P.bit_words);
    if (rc2) return rc2;
    P.layout = integer;
    for (uint32_t a = 0; a < A; a++) q.aggs[a] = P.aggs[a];
  }
  for (uint32_t k = 0; k < K; k++) projected.insert(plan->keys[k].col_id & ~PG_COL_DERIVED);
  for (uint32_t a = 0; a < A; a++) q.agg_reads |= plan->aggs[a].fn != PG_AGG_COUNT;

  PG_PROF("state");
  // ---- group state addressing: dense key space, hash table of global keys, or (numGroupsLimit can truncate a
  // segment) hash table of (segment, key) with first-seen docs
  const uint64_t slot_bytes = 8ull * (P.n_i64 + 2ull * P.n_fx + P.n_min + P.n_max) + 4ull * P.bit_words;
  if (K == 0) {
    P.mode = GM_NONE;
    P.num_slots = 1;
  } else {
    const bool dense = !(plan->flags & PG_PLAN_HASH_GROUPS) && G <= kDenseMaxSlots &&
                       G * slot_bytes <= kStateBudget / 4 && G <= 4 * (t_layout.on ? t_layout.docs : total_docs) + 65536;
    // numGroupsLimit truncation assigns ids in first-seen (doc, key tuple) order: the per-segment table's sort key
    // packs (segment, doc, tuple position) into 16 + 32 + 16 bits for multi-value keys
    if (truncating && q.mv_keys && S > 0xFFFFu)
      return fail(PG_E_UNSUPPORTED, "multi-value group keys under numGroupsLimit over more than 65535 segments in one call");
    P.mode = truncating ? GM_HASH_SEG : (dense ? GM_DENSE : GM_HASH);
    if (P.mode == GM_DENSE) {
      P.num_slots = G;
    } else {
      if (P.mode == GM_HASH_SEG && (G - 1) > ((1ull << 62) - S) / std::max(1u, S))
        return fail(PG_E_UNSUPPORTED, "per-segment group key (key space %llu x %u segments) exceeds 62 bits",
                    (unsigned long long)G, S);
      const uint64_t expect = P.mode == GM_HASH_SEG ? seg_groups : std::min(G, std::min(total_docs, seg_groups));
      uint64_t cap = hash_cap ? hash_cap : pow2_at_least(std::max<uint64_t>(1024, 2 * expect));
      // large bounds start smaller and grow on overflow (err bit 4 -> rerun with 8x the table)
      if (!hash_cap && cap * (slot_bytes + 12) > (4ull << 30)) cap = std::max<uint64_t>(1024, pow2_at_least((4ull << 30) / (slot_bytes + 12)) / 2);
      if (cap > kMaxHashSlots || cap * (slot_bytes + 12) > kStateBudget)
        return fail(PG_E_UNSUPPORTED, "group-by hash table of %llu slots x %llu bytes exceeds the state budget",
                    (unsigned long long)cap, (unsigned long long)slot_bytes);
      P.num_slots = cap;
      P.max_fill = (uint32_t)(cap / 4 * 3);
    }
  }
  if (P.num_slots * slot_bytes > kStateBudget)
    return fail(PG_E_UNSUPPORTED, "group state of %llu bytes exceeds the budget", (unsigned long long)(P.num_slots * slot_bytes));
  q.group_mode = P.mode;
  q.num_slots = P.num_slots;
  q.hmask = P.mode == GM_HASH || P.mode == GM_HASH_SEG ? P.num_slots - 1 : 0;
  q.hmax_fill = P.max_fill;
  q.n_i64 = P.n_i64; q.n_fx = P.n_fx; q.n_min = P.n_min; q.n_max = P.n_max;
  q.dc_row_words = P.bit_words;
  // aggregation-only plans with SK_FX sums use a one-slot LDS table for them (pg_scan.hip acc_update)
  q.use_lds = (P.mode == GM_DENSE || (P.mode == GM_NONE && P.n_fx)) &&
              P.num_slots * 8ull * (P.n_i64 + 2ull * P.n_fx + P.n_min + P.n_max) <= (uint64_t)kLdsGroupBytes;
  // ---- radix-partitioned dense group-by (pg_part.hip) for a dense key space whose state is far larger than any
  // cache, when the aggregations are COUNTs and at most one DISTINCTCOUNT (entries of key low bits | value id fit 32
  // bits).  PG_PART=0|1 overrides the size threshold.
  PartPlan part;
  {
    const char* part_env = getenv("PG_PART");
    const int pe = part_env ? atoi(part_env) : -1;
    uint32_t dc = (uint32_t)kNoSlot, ndc = 0;
    bool ok = P.mode == GM_DENSE && !q.use_lds && K > 0 && P.n_i64 == 1 && !P.n_fx && !P.n_min && !P.n_max &&
              total_docs > 0 && total_docs < 0xFFFFFFF0ull && pe != 0 && !q.mv_keys && !q.mv_aggs;
    for (uint32_t a = 0; a < A && ok; a++) {
      if (P.aggs[a].fn == PG_AGG_DISTINCTCOUNT) { dc = a; ndc++; }
      else if (P.aggs[a].fn != PG_AGG_COUNT) ok = false;
    }
    ok = ok && ndc <= 1 && (pe == 1 || G * slot_bytes >= kPartMinStateBytes);
    if (ok) {
      auto clog2 = [](uint64_t x) { uint32_t b = 0; while ((1ull << b) < x) b++; return b; };
      const uint32_t gbits = clog2(G);
      static const uint32_t l1_bits = getenv("PG_PART_L1_BITS") ? (uint32_t)std::min(std::max(atoi(getenv("PG_PART_L1_BITS")), 1), 8) : 8u;
      part.shift1 = gbits > l1_bits ? gbits - l1_bits : 0;
      part.vbits = dc == (uint32_t)kNoSlot ? 0 : clog2(P.aggs[dc].key_card);
      part.dc_words = dc == (uint32_t)kNoSlot ? 0 : (P.aggs[dc].key_card + 31) / 32;
      const uint64_t per_group = 4ull * (1 + part.dc_words);
      uint32_t sh2 = 0;
      while ((per_group << (sh2 + 1)) <= (uint64_t)kPartLdsBytes) sh2++;
      part.shift2 = std::min(sh2, part.shift1);
      if (per_group <= (uint64_t)kPartLdsBytes && part.shift1 + part.vbits <= 32 && part.vbits < 32 &&
          part.shift1 - part.shift2 <= 8 && gbits + part.vbits <= 64) {
        part.on = true;
        part.dc = dc;
        part.dc_word = dc == (uint32_t)kNoSlot ? 0 : P.aggs[dc].dc_word;
        part.nparts1 = (uint32_t)(((G - 1) >> part.shift1) + 1);
        part.nparts2 = 1u << (part.shift1 - part.shift2);
      }
    }
  }
  P.projected_cols = (uint32_t)projected.size();
  P.total_docs = total_docs;
  P.num_segments = S;

  PG_PROF("sets");
  // ---- per (segment, leaf) lowering.  A leaf's dictId set becomes: a contiguous range -> RANGE; a small set
  // -> LDS hash set (uniform table size per leaf across segments so the LDS layout is fixed); else a global
  // bitmap over dictIds built on the device (one batched launch).
  // Per leaf: LDS words of its IN-set region (uniform across segments), 0 = gathered through a global LUT.
  // Region = filter bitmap over dictId >> shift (<= 8 KB) + (shift > 0) an exact hash table (<= 50 % full).
  // LDS filter bitmap over dictId >> shift: at most kLdsSetBytes (shift > 0 adds an exact global LUT)
  auto set_geometry = [](uint32_t card, uint32_t& shift, uint32_t& nbw) {
    shift = 0;
    while (((card + (1u << shift) - 1) >> shift) > (uint32_t)(kLdsSetBytes * 8 - 32)) shift++;
    nbw = (((card + (1u << shift) - 1) >> shift) + 31) / 32 + 1;
    return nbw;
  };
  std::vector<uint32_t> set_ints(L, 0), set_off(L, 0);
  std::vector<double> leaf_pass(L, 0.0), leaf_cost(L, 0.0), leaf_reach(L, 0.0);
  double filter_pass = 1.0;
  {
    for (uint32_t si = 0; si < S; si++)
      for (uint32_t li = 0; li < L; li++) {
        const pg_leaf& pl = plan->segments[si].leaves[li];
        if (pl.kind != PG_LEAF_SV_SCAN || pl.num_ids == 0) continue;
        const ColumnRes* c = col(si, pl.col_id);
        if (!c) continue;
        uint32_t sh, nbw;
        set_ints[li] = std::max(set_ints[li], set_geometry(std::max(c->card, 1u), sh, nbw));
      }
    uint32_t used = 0;
    for (uint32_t li = 0; li < L; li++) {
      if (!set_ints[li] || pl_too_big(set_ints[li]) || (used + set_ints[li]) * 4ull > (uint64_t)kLdsSetBytes) {
        set_ints[li] = 0;
        continue;
      }
      set_off[li] = used;
      used += (set_ints[li] + 3) & ~3u;
    }
    q.set_lds_ints = used;
  }
  // pass-fraction / cost estimates (averaged over segments) for the AND / OR child order
  for (uint32_t si = 0; si < S; si++) {
    const double w = 1.0 / S;
    for (uint32_t li = 0; li < L; li++) {
      const pg_leaf& pl = plan->segments[si].leaves[li];
      const ColumnRes* c = (pl.kind == PG_LEAF_MATCH_ALL || pl.kind == PG_LEAF_EMPTY) ? nullptr : col(si, pl.col_id);
      double f = 1.0, cost = 0.0;
      if (pl.kind == PG_LEAF_EMPTY) f = 0.0;
      else if (c && pl.kind == PG_LEAF_RAW_SCAN) {
        // uniform over [min, max] for a range, distinct values ~ cardinality for a set
        if (pl.num_ids) f = std::min(1.0, pl.num_ids / (double)std::max(1u, c->card));
        else {
          const double lo = c->dtype <= PG_LONG ? (double)pl.ilo : pl.dlo, hi = c->dtype <= PG_LONG ? (double)pl.ihi : pl.dhi;
          const double span = c->dmax - c->dmin;
          f = span > 0 ? std::max(0.0, std::min(1.0, (std::min(hi, c->dmax) - std::max(lo, c->dmin)) / span)) : 1.0;
        }
        if (pl.exclusive) f = 1.0 - f;
        cost = c->dtype == PG_INT || c->dtype == PG_FLOAT ? 4.0 : 8.0;
      } else if (c) {
        const double card = std::max(1u, c->card);
        const double nset = pl.num_ids ? pl.num_ids : std::max(0, std::min(pl.hi, (int32_t)c->card) - std::max(pl.lo, 0));
        f = std::min(1.0, nset / card);
        if (pl.exclusive) f = 1.0 - f;
        if (pl.kind == PG_LEAF_SV_SCAN) cost = c->bits / 8.0;
        if (pl.kind == PG_LEAF_RANGE_INDEX) cost = c->vbits / 8.0;
        if (pl.kind == PG_LEAF_MV_SCAN) cost = 0.0;  // materialised by the pre-pass
      }
      leaf_pass[li] += w * f;
      leaf_cost[li] += w * cost;
    }
  }
  PG_PROF("order");
  // ---- streaming pre-filter (pg_filter.hip): the leaf children of a root AND (or a lone leaf) whose joint pass
  // fraction is small are evaluated by lean per-bit-width kernels into one doc bitmap per segment; the fused scan
  // then sees that bitmap as ONE 1-bit leaf and the other folded leaves as match-all.  Opt-in (PG_PREFILTER=1):
  // measured slower than the fused scan alone on configs 2 and 3 (r02_v1: config 2 step 1.19 ->
  // 1.90 ms, config 3 1.54 -> 2.80 ms), because the fused scan's short-circuit already skips most bytes.
  std::vector<uint32_t> pre_leaves;
  {
    std::vector<FNode> nodes;
    int root = -1;
    build_tree(plan, leaf_pass, leaf_cost, nodes, root);
    if (root >= 0) {
      const char* pf_env = getenv("PG_PREFILTER");
      const int pf = pf_env ? atoi(pf_env) : -1;
      std::vector<int> kids;
      if (nodes[root].kind == 0) kids.push_back(root);
      else if (nodes[root].kind == 1) kids = nodes[root].kids;
      double pass = 1.0, cost = 0.0;
      std::vector<uint32_t> cand;
      for (int k : kids)
        if (nodes[k].kind == 0) {
          cand.push_back((uint32_t)nodes[k].leaf);
          pass *= leaf_pass[nodes[k].leaf];
          cost += leaf_cost[nodes[k].leaf];
        }
      bool raw_leaf = false;
      for (uint32_t li : cand)
        for (uint32_t si = 0; si < S; si++) raw_leaf |= plan->segments[si].leaves[li].kind == PG_LEAF_RAW_SCAN;
      if (!cand.empty() && pf == 1 && !raw_leaf) {
        pre_leaves = cand;
        leaf_pass[cand[0]] = pass;
        leaf_cost[cand[0]] = 1.0 / 8;
        for (size_t i = 1; i < cand.size(); i++) { leaf_pass[cand[i]] = 1.0; leaf_cost[cand[i]] = 0.0; }
        nodes.clear();
        build_tree(plan, leaf_pass, leaf_cost, nodes, root);
      }
    }
    std::vector<int32_t> pre;
    if (root >= 0) {
      emit_prefix(nodes, root, pre);
      assign_reach(nodes, root, 1.0, leaf_reach);
      filter_pass = nodes[root].pass;
    }
    if (pre.size() > (size_t)kMaxOps) return fail(PG_E_UNSUPPORTED, "filter program longer than %d", kMaxOps);
    int depth = 0, md = 0;
    for (int32_t op : pre) {
      if (op == kOpAnd || op == kOpOr || op == kOpNot) md = std::max(md, ++depth);
      else if (op == kOpEnd) depth--;
    }
    if (md > kMaxDepth) return fail(PG_E_UNSUPPORTED, "filter nesting deeper than %d", kMaxDepth);
    q.num_ops = (uint32_t)pre.size();
    for (size_t i = 0; i < pre.size(); i++) q.ops[i] = pre[i];
  }

  Arena ar(t_ctx.arena);
  std::vector<LeafDesc> leaves((uint64_t)S * L);
  std::vector<ColDesc> aggcols((uint64_t)S * A * 2);
  std::vector<ColDesc> keycols((uint64_t)S * K);
  std::vector<SegDesc> segd(S);
  std::vector<WorkItem>& items = t_ctx.items;
  items.clear();
  std::vector<PrepassOp> pre;
  struct LutReq {  // arena ids (or literal values found in `dict`) -> scratch LUT and / or LDS-set region (~0 = none)
    uint64_t ids_off; uint32_t n; uint64_t lut_off; uint64_t region_off = ~0ull; uint32_t shift = 0;
    uint64_t vals_off = ~0ull; const void* dict = nullptr; uint32_t card = 0, dtype = 0;
  };
  std::vector<LutReq> luts;
  // values-mode leaves (pg_leaf.num_values): each literal list once in the arena per (host pointer, stored type)
  std::map<std::pair<const void*, uint32_t>, uint64_t> lit_arena;
  auto literals_off = [&](const pg_leaf& pl, uint32_t dtype) -> uint64_t {
    auto it = lit_arena.find({pl.values, dtype});
    if (it != lit_arena.end()) return it->second;
    const uint32_t n = pl.num_values, w = dtype == PG_INT || dtype == PG_FLOAT ? 4 : 8;
    const uint64_t at = ar.reserve((uint64_t)w * n);
    for (uint32_t i = 0; i < n; i++) {
      uint8_t* dst = &ar.h[at + (uint64_t)w * i];
      if (dtype == PG_INT) { const int32_t v = (int32_t)((const int64_t*)pl.values)[i]; memcpy(dst, &v, 4); }
      else if (dtype == PG_LONG) memcpy(dst, (const int64_t*)pl.values + i, 8);
      else if (dtype == PG_FLOAT) { const float v = (float)((const double*)pl.values)[i]; memcpy(dst, &v, 4); }
      else memcpy(dst, (const double*)pl.values + i, 8);
    }
    lit_arena[{pl.values, dtype}] = at;
    return at;
  };
  auto lut_req = [&](const pg_leaf& pl, const ColumnRes* c, uint64_t lut_off, uint64_t region_off, uint32_t shift) {
    LutReq r;
    r.lut_off = lut_off;
    r.region_off = region_off;
    r.shift = shift;
    if (pl.ids) {
      r.ids_off = ar.put(pl.ids, 4ull * pl.num_ids);
      r.n = pl.num_ids;
    } else {  // values mode: the device finds the literals' dictIds
      r.ids_off = ~0ull;
      r.vals_off = literals_off(pl, c->dtype);
      r.n = pl.num_values;
      r.dict = c->dict.p;
      r.card = c->card;
      r.dtype = c->dtype;
    }
    luts.push_back(r);
  };
  // a leaf's dictId list in the arena, shared with the previous segment's when byte-identical (segments of one table
  // whose dictionaries agree lower an IN list to the same ids: config 5's 32 segments x 2 022 ids = 0.26 MB of arena
  // the device would otherwise read over the host link); the lists are only read on the device
  struct LastIds { const int32_t* src = nullptr; uint32_t n = 0; uint64_t off = 0; };
  std::vector<LastIds> last_ids(L);  // per leaf: the previous segment's list (caller memory, live for the call)
  auto put_ids = [&](uint32_t li, const int32_t* ids, uint32_t n) -> uint64_t {
    LastIds& x = last_ids[li];
    if (x.src && n && x.n == n && (x.src == ids || memcmp(x.src, ids, 4ull * n) == 0)) return x.off;
    x = {ids, n, ar.put(ids, 4ull * n)};
    return x.off;
  };
  uint64_t scratch_bytes = 0;
  auto scratch_reserve = [&](uint64_t n) { uint64_t at = (scratch_bytes + 255) & ~255ull; scratch_bytes = at + n; return at; };
  // LK_SET_LDS leaves: their coarse filter bitmap (region) and exact LUT, reserved in scratch once the stream plan is
  // known -- a segment whose driving IN leaf the exact-mode stream tests builds that leaf's LUT in LDS from its dictIds
  // and needs neither (nor their zero fill and set_lut_bits job)
  struct SetLdsRes { uint64_t leaf_index; size_t lut_req; uint64_t region_bytes, lut_bytes; };
  std::vector<SetLdsRes> set_lds_res;
  uint64_t entries_in_filter = 0;
  // device pointers into arena / scratch are patched once those are allocated
  enum PatchTarget { PT_AUX = 0, PT_WORDS = 1, PT_LUT = 2, PT_RVALS = 3 };
  struct Patch { uint64_t leaf_index; uint64_t off; bool in_arena; int target; bool orig = false; };
  std::vector<Patch> patches;

  PG_PROF("nonscan");
  // ---- NonScanBasedAggregationOperator route (plan/AggregationPlanNode.java:185-197, :236-261): with no group-by,
  // a segment whose filter matches all docs and functions that are COUNT or MIN / MAX / DISTINCTCOUNT of a column
  // with a dictionary is answered from its dictionary instead of scanned (ExecutionStatistics(numTotalDocs, 0, 0,
  // numTotalDocs), NonScanBasedAggregationOperator.java:253-256).  PG_NONSCAN=0 scans them instead.
  std::vector<uint8_t> nonscan(S, 0);
  uint64_t ns_docs = 0, ns_matched = 0;
  {
    const char* ns_env = getenv("PG_NONSCAN");
    bool fit = K == 0 && !(ns_env && atoi(ns_env) == 0);
    for (uint32_t a = 0; a < A && fit; a++) {
      const pg_agg& g = plan->aggs[a];
      if (g.fn == PG_AGG_COUNT) continue;
      fit = (g.fn == PG_AGG_MIN || g.fn == PG_AGG_MAX || g.fn == PG_AGG_DISTINCTCOUNT) && g.op == PG_EXPR_COL;
    }
    for (uint32_t si = 0; si < S && fit; si++) {
      bool ok = filter_is_match_all(plan, plan->segments[si].leaves);
      for (uint32_t a = 0; a < A && ok; a++) {
        const pg_agg& g = plan->aggs[a];
        if (g.fn == PG_AGG_COUNT) continue;
        const ColumnRes* c = col(si, g.col_a);
        // MIN / MAX: dictionary or column metadata (a raw column's min / max); DISTINCTCOUNT: the dictionary
        ok = c && ((c->has_dict && c->dict.p) || (c->fwd == FWD_RAW && g.fn != PG_AGG_DISTINCTCOUNT)) &&
             (g.fn != PG_AGG_DISTINCTCOUNT || g.key_kind != PG_KEY_KEYMAP || c->has_keymap);
      }
      if (!ok) continue;
      nonscan[si] = 1;
      ns_docs += plan->segments[si].num_docs;
      ns_matched += plan->segments[si].num_docs > 0;
    }
  }

  std::vector<uint32_t> seg_tiles(S, 0);
  for (uint32_t si = 0; si < S; si++) {
    const pg_segment_ref& sr = plan->segments[si];
    segd[si].num_docs = sr.num_docs;
    segd[si].index = si;
    seg_tiles[si] = nonscan[si] ? 0u : (uint32_t)(((uint64_t)sr.num_docs + kTileDocs - 1) / kTileDocs);
    for (uint32_t li = 0; li < L; li++) {
      const pg_leaf& pl = sr.leaves[li];
      LeafDesc& dl = leaves[(uint64_t)si * L + li];
      memset(&dl, 0, sizeof(dl));
      dl.excl = pl.exclusive ? 1 : 0;
      if (pl.kind == PG_LEAF_MATCH_ALL) { dl.kind = LK_ALL; dl.excl = 0; continue; }
      if (pl.kind == PG_LEAF_EMPTY) { dl.kind = LK_NONE; dl.excl = 0; continue; }
      const ColumnRes* c = col(si, pl.col_id);
      if (!c) return fail(PG_E_NOTFOUND, "leaf %u: column %u not resident in segment %u", li, pl.col_id, si);
      if (pl.kind == PG_LEAF_RAW_SCAN) {
        // raw-value predicate over a raw forward index: values gathered per needed doc, compared in their type
        if (c->fwd != FWD_RAW) return fail(PG_E_INVALID, "raw leaf on column %u without a raw forward index", pl.col_id);
        if (c->num_docs < sr.num_docs) return fail(PG_E_INVALID, "column %u has %u docs < segment's %u", pl.col_id, c->num_docs, sr.num_docs);
        if (pl.num_ids && !pl.values) return fail(PG_E_INVALID, "leaf %u: null value list", li);
        dl.kind = LK_RAW;
        dl.words = (const uint32_t*)c->rawv.p;
        dl.rtype = c->dtype;
        dl.ilo = pl.ilo; dl.ihi = pl.ihi; dl.dlo = pl.dlo; dl.dhi = pl.dhi;
        dl.rflags = (pl.lo_inclusive ? 1u : 0u) | (pl.hi_inclusive ? 2u : 0u);
        dl.nvals = pl.num_ids;
        if (pl.num_ids) {  // int64 (INT / LONG) or double (FLOAT / DOUBLE), sorted: binary search on the device
          const uint64_t off = ar.put(pl.values, 8ull * pl.num_ids);
          patches.push_back({(uint64_t)si * L + li, off, true, PT_RVALS});
        }
        if (!index_leaf[(uint64_t)si * L + li]) entries_in_filter += sr.num_docs;
        continue;
      }
      if (pl.kind == PG_LEAF_RANGE_INDEX) {  // raw INT / LONG range index: offsets [lo, hi) of the packed values
        dl.kind = LK_RANGE;
        dl.words = (const uint32_t*)c->vals.p;
        dl.wbytes = (uint32_t)std::min<uint64_t>(c->vals.bytes, 0xFFFFFFF0ull);
        dl.bits = c->vbits;
        dl.lo = pl.lo;
        dl.hi = std::max(pl.hi, pl.lo);
        continue;
      }
      // values mode (pg_leaf.num_values): the literals themselves, for SV / MV scans over a resident dictionary
      const bool vmode = pl.num_ids && !pl.ids && pl.num_values;
      if (vmode && (!pl.values || (pl.kind != PG_LEAF_SV_SCAN && pl.kind != PG_LEAF_MV_SCAN) || !c->has_dict ||
                    !c->dict.p || c->dtype > PG_DOUBLE))
        return fail(PG_E_INVALID, "leaf %u: literal values need an SV / MV scan over a numeric dictionary", li);
      if (pl.num_ids && !pl.ids && !vmode) return fail(PG_E_INVALID, "leaf %u: null id list", li);
      if (!vmode && !ids_valid(pl.ids, pl.num_ids, std::max(c->card, 1u)))
        return fail(PG_E_INVALID, "leaf %u: dictIds must be sorted, unique and < cardinality", li);
      auto in_set = [&](int32_t id) {
        if (!pl.num_ids) return id >= pl.lo && id < pl.hi;
        return std::binary_search(pl.ids, pl.ids + pl.num_ids, id);
      };
      switch (pl.kind) {
        case PG_LEAF_SV_SCAN: {
          if (c->fwd != FWD_SV && c->fwd != FWD_SORTED) return fail(PG_E_INVALID, "SV scan on column %u without SV forward index", pl.col_id);
          if (c->num_docs < sr.num_docs) return fail(PG_E_INVALID, "column %u has %u docs < segment's %u", pl.col_id, c->num_docs, sr.num_docs);
          dl.words = (const uint32_t*)c->words.p;
          dl.wbytes = (uint32_t)std::min<uint64_t>(c->words.bytes, 0xFFFFFFF0ull);
          dl.bits = c->bits;
          if (!index_leaf[(uint64_t)si * L + li]) entries_in_filter += sr.num_docs;
          const bool contiguous = !vmode && pl.num_ids && (uint32_t)(pl.ids[pl.num_ids - 1] - pl.ids[0]) + 1 == pl.num_ids;
          if (!pl.num_ids || contiguous) {
            dl.kind = LK_RANGE;
            const int32_t lo = pl.num_ids ? pl.ids[0] : pl.lo, hi = pl.num_ids ? pl.ids[pl.num_ids - 1] + 1 : pl.hi;
            dl.lo = std::max(lo, 0);
            dl.hi = std::max(std::min(hi, (int32_t)c->card), dl.lo);
          } else if (set_ints[li]) {
            dl.kind = LK_SET_LDS;
            const uint32_t n_region = set_geometry(std::max(c->card, 1u), dl.shift, dl.nbw);
            dl.set_ints = n_region;
            dl.lds_off = set_off[li];
            // filter bitmap (and, when shift > 0, the exact LUT resolving its candidates) built on the device, in
            // scratch reserved once the stream plan is known (set_lds_res)
            set_lds_res.push_back({(uint64_t)si * L + li, luts.size(), 4ull * n_region,
                                   dl.shift ? 4ull * ((c->card + 31) / 32 + 1) : 0ull});
            lut_req(pl, c, ~0ull, ~0ull, dl.shift);
          } else {
            dl.kind = LK_SET_LUT;
            const uint64_t lut_off = scratch_reserve(4ull * ((c->card + 31) / 32 + 1));
            lut_req(pl, c, lut_off, ~0ull, 0);
            patches.push_back({(uint64_t)si * L + li, lut_off, false, PT_AUX});
          }
          break;
        }
        case PG_LEAF_SORTED: {
          if (c->fwd != FWD_SORTED) return fail(PG_E_INVALID, "sorted leaf on unsorted column %u", pl.col_id);
          // SortedIndexBasedFilterOperator: matching dictIds -> merged [start,end] doc ranges
          // (a sorted column's docs are ordered by dictId, so only the selected ids are visited: a dictId range is
          // one doc range from its first to its last non-empty id)
          std::vector<int32_t> rg;
          auto add_id = [&](int32_t id) {
            const int32_t s0 = c->sorted_pairs[2 * id], e0 = std::min(c->sorted_pairs[2 * id + 1], (int32_t)sr.num_docs - 1);
            if (e0 < s0) return;
            if (!rg.empty() && rg.back() + 1 >= s0) rg.back() = std::max(rg.back(), e0);
            else { rg.push_back(s0); rg.push_back(e0); }
          };
          if (pl.num_ids) {
            for (uint32_t i = 0; i < pl.num_ids; i++) add_id(pl.ids[i]);
          } else {
            int32_t lo = std::max(pl.lo, 0), hi = std::min(pl.hi, (int32_t)c->card);
            auto empty = [&](int32_t id) { return std::min(c->sorted_pairs[2 * id + 1], (int32_t)sr.num_docs - 1) < c->sorted_pairs[2 * id]; };
            while (lo < hi && empty(lo)) lo++;
            while (hi > lo && empty(hi - 1)) hi--;
            if (lo < hi) {
              rg.push_back(c->sorted_pairs[2 * lo]);
              rg.push_back(std::min(c->sorted_pairs[2 * (hi - 1) + 1], (int32_t)sr.num_docs - 1));
            }
          }
          if (pl.exclusive) {  // complement within [0, num_docs)
            std::vector<int32_t> cm;
            int32_t next = 0;
            for (size_t i = 0; i < rg.size(); i += 2) {
              if (rg[i] > next) { cm.push_back(next); cm.push_back(rg[i] - 1); }
              next = rg[i + 1] + 1;
            }
            if (next < (int32_t)sr.num_docs) { cm.push_back(next); cm.push_back((int32_t)sr.num_docs - 1); }
            rg.swap(cm);
          }
          dl.excl = 0;
          if (rg.empty()) { dl.kind = LK_NONE; break; }
          if (rg.size() == 2) { dl.kind = LK_DOCRANGE; dl.lo = rg[0]; dl.hi = rg[1] + 1; break; }
          as_bitmap_leaf(dl, sr.num_docs);
          PrepassOp op{PrepassOp::FILL_RANGES, si, li};
          op.in_off = ar.put(rg.data(), 4ull * rg.size());
          op.n = (uint32_t)(rg.size() / 2);
          op.num_docs = sr.num_docs;
          op.out_off = scratch_reserve(4ull * ((sr.num_docs + 31) / 32 + 1));
          patches.push_back({(uint64_t)si * L + li, op.out_off, false, PT_WORDS});
          pre.push_back(op);
          break;
        }
        case PG_LEAF_INVERTED: {
          if (!c->has_inv) return fail(PG_E_INVALID, "inverted leaf on column %u without inverted index", pl.col_id);
          as_bitmap_leaf(dl, sr.num_docs);
          dl.excl = 0;
          PrepassOp op{PrepassOp::ROARING, si, li};
          if (pl.num_ids) {  // the selected dictIds; the device finds their containers per 64 K-doc key
            op.in_off = put_ids(li, pl.ids, pl.num_ids);
            op.n = pl.num_ids;
          } else {
            const int32_t lo = std::max(pl.lo, 0), hi = std::max(std::min(pl.hi, (int32_t)c->card), lo);
            const uint64_t at = ar.reserve(4ull * (uint32_t)(hi - lo));
            for (int32_t id = lo; id < hi; id++) memcpy(&ar.h[at + 4ull * (uint32_t)(id - lo)], &id, 4);
            op.in_off = at;
            op.n = (uint32_t)(hi - lo);
          }
          op.key0 = 0;
          op.nkeys = (sr.num_docs + 65535) >> 16;
          op.num_docs = sr.num_docs;
          op.col = c;
          op.negate = pl.exclusive != 0;
          op.out_off = scratch_reserve(4ull * ((sr.num_docs + 31) / 32 + 1));
          patches.push_back({(uint64_t)si * L + li, op.out_off, false, PT_WORDS});
          pre.push_back(op);
          break;
        }
        case PG_LEAF_MV_SCAN: {
          if (c->fwd != FWD_MV) return fail(PG_E_INVALID, "MV scan on column %u without MV forward index", pl.col_id);
          entries_in_filter += c->num_values;
          as_bitmap_leaf(dl, sr.num_docs);
          dl.excl = 0;
          PrepassOp op{PrepassOp::MV_SCAN, si, li};
          op.col = c;
          op.num_docs = sr.num_docs;
          op.excl = pl.exclusive ? 1 : 0;
          op.lo = pl.lo;
          op.hi = pl.hi;
          if (pl.num_ids) {
            op.lut_off = scratch_reserve(4ull * ((c->card + 31) / 32 + 1));
            lut_req(pl, c, op.lut_off, ~0ull, 0);
          }
          op.out_off = scratch_reserve(4ull * ((sr.num_docs + 31) / 32 + 1));
          patches.push_back({(uint64_t)si * L + li, op.out_off, false, PT_WORDS});
          pre.push_back(op);
          break;
        }
        default:
          return fail(PG_E_INVALID, "unknown leaf kind %u", pl.kind);
      }
    }
    for (uint32_t li = 0; li < L && li < PG_TRACE_MAX_LEAVES; li++)  // the trace: the form each leaf took here
      t_trace.leaf_forms[li][leaf_form(sr.leaves[li], leaves[(uint64_t)si * L + li])]++;
    for (uint32_t a = 0; a < A; a++) {
      const pg_agg& g = plan->aggs[a];
      if (g.fn == PG_AGG_COUNT) continue;
      const uint32_t cids[2] = {g.col_a, g.col_b};
      const int n = (g.op != PG_EXPR_COL && g.fn != PG_AGG_DISTINCTCOUNT && g.fn != PG_AGG_COUNTMV) ? 2 : 1;
      for (int k = 0; k < n; k++) {
        const ColumnRes* c = col(si, cids[k]);
        if (c->num_docs < sr.num_docs) return fail(PG_E_INVALID, "column %u has %u docs < segment's %u", cids[k], c->num_docs, sr.num_docs);
        ColDesc& dc = aggcols[((uint64_t)si * A + a) * 2 + k];
        dc.words = (const uint32_t*)c->words.p;
        dc.wbytes = (uint32_t)std::min<uint64_t>(c->words.bytes, 0xFFFFFFF0ull);
        dc.dict = c->dict.p;
        dc.keymap = (const int32_t*)c->keymap.p;
        dc.mv_offsets = (const uint32_t*)c->mv_offsets.p;
        dc.bits = c->bits;
        dc.dtype = c->dtype;
        dc.card = c->card;
        if (c->fwd == FWD_RAW && agg_decodes(g) && c->vals.p) {
          use_decoded(dc, c);  // the range index's packed (value - min) offsets: fewer bytes than the values
        } else if (c->fwd == FWD_RAW) {  // the values themselves: "dictId" = doc id (bits 0), "dictionary" = the values
          dc.words = nullptr;
          dc.wbytes = 0;
          dc.bits = 0;
          dc.dict = c->rawv.p;
          dc.card = c->num_docs;
        } else if (agg_decodes(g) && (c->vals.p || c->identity)) {
          use_decoded(dc, c);
        }
      }
    }
    for (uint32_t k = 0; k < K; k++) {
      const ColumnRes* c = col(si, plan->keys[k].col_id);
      if (c->num_docs < sr.num_docs) return fail(PG_E_INVALID, "key column %u has fewer docs than the segment", plan->keys[k].col_id);
      key_coldesc(keycols[(uint64_t)si * K + k], c, plan->keys[k]);
    }
  }
  P.entries_in_filter = entries_in_filter;
  // The docs that can match at all: the doc ranges among the root AND's direct children (sorted-index leaves; an
  // empty leaf empties it).  They bound the 64 K-doc keys an inverted leaf's roaring pre-pass builds and the tiles
  // the fused scan walks (SortedIndexBasedFilterOperator + AndDocIdSet: the other children are only asked about docs
  // inside the range).
  std::vector<std::pair<uint32_t, uint32_t>> root_range(S);
  {
    std::vector<int> root_leaves;  // direct leaf children of the root AND (postfix: the operands on the stack)
    if (plan->num_ops == 1 && plan->ops[0] >= 0) {
      root_leaves.push_back(plan->ops[0]);  // a lone leaf
    } else if (plan->num_ops && plan->ops[plan->num_ops - 1] < 0 && ((-plan->ops[plan->num_ops - 1]) & 0x300) == 0x100) {
      std::vector<int> st;  // stack of leaf index or -1 (a subtree)
      for (uint32_t i = 0; i < plan->num_ops; i++) {
        const int32_t op = plan->ops[i];
        if (op >= 0) { st.push_back(op); continue; }
        const int n = op == PG_OP_NOT ? 1 : ((-op) & 0xFF);
        if (i + 1 == plan->num_ops) root_leaves.assign(st.end() - n, st.end());
        st.resize(st.size() - n);
        st.push_back(-1);
      }
    }
    for (uint32_t si = 0; si < S; si++) {
      int64_t lo = 0, hi = plan->segments[si].num_docs;
      for (int li : root_leaves) {
        if (li < 0) continue;
        const LeafDesc& dl = leaves[(uint64_t)si * L + li];
        if (dl.kind == LK_DOCRANGE) { lo = std::max<int64_t>(lo, dl.lo); hi = std::min<int64_t>(hi, dl.hi); }
        else if (dl.kind == LK_NONE) hi = lo;
      }
      root_range[si] = hi > lo ? std::make_pair((uint32_t)lo, (uint32_t)hi) : std::make_pair(0u, 0u);
    }
  }
  for (PrepassOp& op : pre) {
    if (op.kind != PrepassOp::ROARING) continue;
    const uint32_t lo = root_range[op.seg].first, hi = std::min(root_range[op.seg].second, op.num_docs);
    if (hi <= lo) { op.nkeys = 0; continue; }
    op.key0 = lo >> 16;
    op.nkeys = ((hi - 1) >> 16) + 1 - op.key0;
  }
  // the fused scan's tiles of each segment: those overlapping its root range
  std::vector<uint32_t> seg_tile0(S, 0);
  for (uint32_t si = 0; si < S; si++) {
    if (!seg_tiles[si]) continue;
    const uint32_t lo = root_range[si].first, hi = root_range[si].second;
    if (hi <= lo) { seg_tiles[si] = 0; continue; }
    seg_tile0[si] = lo / kTileDocs;
    seg_tiles[si] = (hi + kTileDocs - 1) / kTileDocs - seg_tile0[si];
  }

  PG_PROF("leaves");
  // ---- pre-filter launches: per folded leaf (in order), one launch per bit width its segments read (doc ranges
  // and constants ride along as width 1); the fused scan's leaf list gets the bitmap leaf + match-all in their place,
  // while the pre-filter reads the original descriptors (leaves_orig, patched like the others)
  struct PreLaunch { uint32_t leaf, bits, first, n_items, set_ints; uint64_t items_off; };
  std::vector<PreLaunch> pre_launches;
  std::vector<LeafDesc> leaves_orig;
  std::vector<uint64_t> pre_bitmap_off(pre_leaves.empty() ? 0 : S);
  if (!pre_leaves.empty()) {
    leaves_orig = leaves;
    for (uint32_t si = 0; si < S; si++)
      pre_bitmap_off[si] = scratch_reserve(4ull * (((uint64_t)plan->segments[si].num_docs + 31) / 32 + 2));
    std::vector<WorkItem> pitems;
    for (size_t k = 0; k < pre_leaves.size(); k++) {
      const uint32_t li = pre_leaves[k];
      std::vector<std::pair<uint32_t, uint32_t>> by_bits;  // (bits, segment)
      for (uint32_t si = 0; si < S; si++) {
        const LeafDesc& dl = leaves[(uint64_t)si * L + li];
        const bool col = dl.kind == LK_RANGE || dl.kind == LK_SET_LDS || dl.kind == LK_SET_LUT;
        by_bits.push_back({col ? dl.bits : 1u, si});
      }
      std::stable_sort(by_bits.begin(), by_bits.end(),
                       [](const std::pair<uint32_t, uint32_t>& a, const std::pair<uint32_t, uint32_t>& b) { return a.first < b.first; });
      for (size_t i = 0; i < by_bits.size();) {
        const uint32_t b = by_bits[i].first;
        pitems.clear();
        uint32_t set_ints = 0;
        for (; i < by_bits.size() && by_bits[i].first == b; i++) {
          const uint32_t si = by_bits[i].second;
          const LeafDesc& dl = leaves[(uint64_t)si * L + li];
          if (dl.kind == LK_SET_LDS) set_ints = std::max(set_ints, dl.lds_off + dl.set_ints);
          const uint32_t groups = (uint32_t)(((uint64_t)plan->segments[si].num_docs + 31) / 32);
          for (uint32_t g0 = 0; g0 < groups; g0 += kPreItemGroups)
            pitems.push_back({si, g0, std::min<uint32_t>(groups, g0 + kPreItemGroups), 0});
        }
        if (pitems.empty()) continue;
        pre_launches.push_back({li, b, k == 0 ? 1u : 0u, (uint32_t)pitems.size(), set_ints,
                                ar.put(pitems.data(), pitems.size() * sizeof(WorkItem))});
      }
    }
    for (Patch& p : patches)
      if (std::find(pre_leaves.begin(), pre_leaves.end(), (uint32_t)(p.leaf_index % L)) != pre_leaves.end()) p.orig = true;
    for (uint32_t si = 0; si < S; si++)
      for (size_t k = 0; k < pre_leaves.size(); k++) {
        LeafDesc& dl = leaves[(uint64_t)si * L + pre_leaves[k]];
        memset(&dl, 0, sizeof(dl));
        if (k == 0) {
          as_bitmap_leaf(dl, plan->segments[si].num_docs);
          patches.push_back({(uint64_t)si * L + pre_leaves[k], pre_bitmap_off[si], false, PT_WORDS});
        } else {
          dl.kind = LK_ALL;
        }
      }
    // the fused scan no longer reads the folded IN sets from LDS
    bool set_lds = false;
    for (const LeafDesc& dl : leaves) set_lds |= dl.kind == LK_SET_LDS;
    if (!set_lds) q.set_lds_ints = 0;
  }
  uint64_t dict_lines = 0;
  for (uint32_t si = 0; si < S; si++) {
    uint64_t seg_lines = 0;
    for (uint32_t a = 0; a < A; a++)
      for (int k = 0; k < 2; k++) {
        const ColDesc& dc = aggcols[((uint64_t)si * A + a) * 2 + k];
        if (dc.dict && dc.bits) seg_lines = std::max<uint64_t>(seg_lines, (uint64_t)dc.card * (dc.dtype == PG_INT || dc.dtype == PG_FLOAT ? 4 : 8) / 128);
      }
    for (uint32_t k = 0; k < K; k++) {
      const ColDesc& dc = keycols[(uint64_t)si * K + k];
      if (dc.dict && plan->keys[k].kind != PG_KEY_KEYMAP)
        seg_lines = std::max<uint64_t>(seg_lines, (uint64_t)dc.card * (dc.dtype == PG_INT || dc.dtype == PG_FLOAT ? 4 : 8) / 128);
    }
    dict_lines = std::max(dict_lines, seg_lines);
  }
  const double decodes = filter_pass * (double)total_docs / std::max(1u, S);
  static const char* xcd_env = getenv("PG_XCD_ORDER");
  bool want_xcd = xcd_env ? atoi(xcd_env) != 0 : (dict_lines >= 2048 && decodes > 16.0 * (double)dict_lines);
  PG_PROF("items");
  // ---- work items.  Balanced form: the concatenated tile sequence of all segments is cut into G equal ranges, one
  // per block, each given as exactly 2 items (split at the segment boundary it crosses, else halved), so the kernel's
  // uniform [2b, 2b + 2) item ranges are tile-exact (+-1 tile per block) and the host emits 2G items instead of one
  // per kItemTiles tiles.  Needs every non-empty segment to hold at least one block's range (so a range crosses at
  // most one boundary); otherwise (and for the XCD-grouped order below, which wants fine items) items of kItemTiles
  // tiles.
  uint32_t grid = 0;
  {
    uint64_t T = 0;
    uint32_t min_tiles = 0xFFFFFFFFu;
    for (uint32_t si = 0; si < S; si++)
      if (seg_tiles[si]) { T += seg_tiles[si]; min_tiles = std::min(min_tiles, seg_tiles[si]); }
    const uint64_t G = std::min<uint64_t>(scan_grid_cap(K > 0), T / 2);
    static const char* bal_env = getenv("PG_BALANCED_ITEMS");
    const bool balanced = (bal_env ? atoi(bal_env) != 0 : !want_xcd) && G >= 1 && (T + G - 1) / G <= min_tiles;
    if (balanced) {
      items.resize(2 * G);
      uint32_t si = 0;
      uint64_t seg_first = 0;  // global index of segment si's first tile
      auto advance = [&](uint64_t t) {  // move si to the segment holding global tile t
        while (!seg_tiles[si] || t >= seg_first + seg_tiles[si]) { seg_first += seg_tiles[si]; si++; }
      };
      // block b's range [b T / G, (b + 1) T / G), the bounds stepped by quotient + remainder (no divisions)
      const uint64_t dq = T / G, dr = T % G;
      uint64_t t1 = 0, rem = 0;
      for (uint64_t b = 0; b < G; b++) {
        const uint64_t t0 = t1;  // >= 2 tiles per block, since G <= T / 2
        t1 += dq;
        rem += dr;
        if (rem >= G) { t1++; rem -= G; }
        advance(t0);
        const uint64_t seg_end = seg_first + seg_tiles[si];
        const uint64_t cut = t1 > seg_end ? seg_end : t0 + (t1 - t0) / 2;
        items[2 * b] = {si, seg_tile0[si] + (uint32_t)(t0 - seg_first), seg_tile0[si] + (uint32_t)(cut - seg_first), 0};
        advance(cut);
        items[2 * b + 1] = {si, seg_tile0[si] + (uint32_t)(cut - seg_first), seg_tile0[si] + (uint32_t)(t1 - seg_first), 0};
      }
      grid = (uint32_t)G;
    } else {
      for (uint32_t s2 = 0; s2 < S; s2++)
        for (uint32_t t = 0; t < seg_tiles[s2]; t += kItemTiles)
          items.push_back({s2, seg_tile0[s2] + t, seg_tile0[s2] + std::min(seg_tiles[s2], t + (uint32_t)kItemTiles), 0});
      // the XCD-grouped order wants every block resident at once (one round), so the step-major interleave holds:
      // dense SUM over a 4 MB dictionary 6.4 ms at 2 rounds -> 4.3 ms at 1 round
      grid = (uint32_t)std::min<uint64_t>(items.size(), scan_grid_cap(K > 0, want_xcd));
    }
  }
  q.num_items = (uint32_t)items.size();

  auto is_pre = [&](uint32_t li) { return std::find(pre_leaves.begin(), pre_leaves.end(), li) != pre_leaves.end(); };
  PG_PROF("staging");
  // ---- staging policy: a packed column is staged per tile (coalesced, every byte used) when the docs the query
  // needs from it are dense enough that a gather would fetch most of its 128-byte lines anyway
  // (reach * docs-per-line >= 1); the rest are gathered per needed doc.  Greedy by reach within the LDS budget.
  {
    struct Cand { uint32_t role, idx, operand; uint64_t key; double reach; uint32_t bmax; };
    std::vector<Cand> cands;
    auto add = [&](uint32_t role, uint32_t idx, uint32_t operand, uint64_t key, double reach, uint32_t bits) {
      for (Cand& c : cands)
        if (c.key == key) { c.reach = std::max(c.reach, reach); c.bmax = std::max(c.bmax, bits); return; }
      cands.push_back({role, idx, operand, key, reach, bits});
    };
    for (uint32_t li = 0; li < L; li++) {
      uint32_t bmax = 0;
      bool bitmap = false, scan = false;
      uint32_t cid = 0;
      for (uint32_t si = 0; si < S; si++) {
        const LeafDesc& dl = leaves[(uint64_t)si * L + li];
        if (dl.kind != LK_RANGE && dl.kind != LK_SET_LDS && dl.kind != LK_SET_LUT) continue;
        bmax = std::max(bmax, dl.bits);
        const pg_leaf& pl = plan->segments[si].leaves[li];
        if (pl.kind == PG_LEAF_SV_SCAN && !is_pre(li)) { scan = true; cid = pl.col_id; } else bitmap = true;
      }
      if (!bmax || (scan && bitmap)) continue;  // mixed per-segment forms: gather
      add(0, li, 0, scan ? (1ull << 32) | cid : (2ull << 32) | li, leaf_reach[li], bmax);
    }
    // aggregation / key uses read the column's decoded forward index in some segment ("decoded" uses: their own
    // slot, key type 3) or dictIds everywhere (key type 1, shared with scan leaves on the column)
    // (an identity dictionary's decoded form IS the dictId stream: it shares the dictIds' slot; an identity
    // ColDesc reads the dictId words, so `words` tells the two decoded forms apart without a column lookup)
    bool agg_dec_v[kMaxAggs][2] = {}, key_dec_v[kMaxKeys] = {};
    for (uint32_t si = 0; si < S; si++) {
      for (uint32_t a = 0; a < A && a < (uint32_t)kMaxAggs; a++)
        for (int k = 0; k < 2; k++) {
          const ColDesc& dc = aggcols[((uint64_t)si * A + a) * 2 + k];
          agg_dec_v[a][k] |= dc.decoded && !dc.identity;
        }
      for (uint32_t k = 0; k < K && k < (uint32_t)kMaxKeys; k++) {
        const ColDesc& dc = keycols[(uint64_t)si * K + k];
        key_dec_v[k] |= dc.decoded && !dc.identity;
      }
    }
    auto agg_dec = [&](uint32_t a, int k) { return agg_dec_v[a][k]; };
    auto key_dec = [&](uint32_t k) { return key_dec_v[k]; };
    for (uint32_t a = 0; a < A; a++) {
      const pg_agg& g = plan->aggs[a];
      if (g.fn == PG_AGG_COUNT || g.fn == PG_AGG_COUNTMV || (g.flags & PG_AGG_MV_VALUES)) continue;
      const int n = (g.op != PG_EXPR_COL && g.fn != PG_AGG_DISTINCTCOUNT) ? 2 : 1;
      for (int k = 0; k < n; k++) {
        const uint32_t cid = k ? g.col_b : g.col_a;
        uint32_t bmax = 0;
        for (uint32_t si = 0; si < S; si++) bmax = std::max(bmax, aggcols[((uint64_t)si * A + a) * 2 + k].bits);
        add(1, a, (uint32_t)k, ((agg_dec(a, k) ? 3ull : 1ull) << 32) | cid, filter_pass, bmax);
      }
    }
    for (uint32_t k = 0; k < K; k++) {
      if ((q.mv_keys >> k) & 1u) continue;  // value-indexed words: read per doc through its row offsets
      uint32_t bmax = 0;
      for (uint32_t si = 0; si < S; si++) bmax = std::max(bmax, keycols[(uint64_t)si * K + k].bits);
      add(2, k, 0, ((key_dec(k) ? 3ull : 1ull) << 32) | plan->keys[k].col_id, filter_pass, bmax);
    }
    std::stable_sort(cands.begin(), cands.end(), [](const Cand& x, const Cand& y) { return x.reach > y.reach; });
    memset(q.leaf_slot, kNoSlot, sizeof(q.leaf_slot));
    memset(q.agg_slot, kNoSlot, sizeof(q.agg_slot));
    memset(q.key_slot, kNoSlot, sizeof(q.key_slot));
    static const char* no_stage = getenv("PG_NO_STAGING");
    // minimum expected needed docs per 128-byte line for staging (PG_STAGE_MIN overrides)
    static const double stage_min = getenv("PG_STAGE_MIN") ? atof(getenv("PG_STAGE_MIN")) : 1.0;
    // LDS bytes of one staging buffer (PG_STAGE_KB overrides kLdsStageBytes)
    static const uint64_t stage_budget = getenv("PG_STAGE_KB") ? 1024ull * (uint64_t)atoi(getenv("PG_STAGE_KB")) : (uint64_t)kLdsStageBytes;
    uint32_t words = 0;
    for (const Cand& c : cands) {
      if (no_stage || q.num_staged >= (uint32_t)kMaxStaged) break;
      if (!c.bmax) continue;  // raw values: read per doc (already consecutive words), never staged
      if (c.reach * 1024.0 / c.bmax < stage_min) continue;
      const uint32_t need = (uint32_t)(kTileDocs / 32) * c.bmax;  // b DMA pieces of 1 KiB
      if ((words + need) * 4ull > stage_budget) continue;
      const uint32_t slot = q.num_staged++;
      q.staged[slot] = {c.role, c.idx, c.operand, words};
      words += need;
      // every use of the same column (in the same form: dictIds or decoded values) shares the slot
      for (uint32_t li = 0; li < L && (c.key >> 32) != 3; li++) {
        bool match = false;
        if ((c.key >> 32) == 2) match = li == (uint32_t)c.key;
        else
          for (uint32_t si = 0; si < S && !match; si++) {
            const pg_leaf& pl = plan->segments[si].leaves[li];
            match = pl.kind == PG_LEAF_SV_SCAN && !is_pre(li) && (uint64_t)pl.col_id == (c.key & 0xFFFFFFFFull) &&
                    leaves[(uint64_t)si * L + li].kind != LK_ALL && leaves[(uint64_t)si * L + li].kind != LK_NONE;
          }
        if (match && (c.key >> 32) == 2) q.leaf_slot[li] = (uint8_t)slot;
        else if (match) {
          // only when every segment's form of this leaf reads the column itself
          bool all_col = true;
          for (uint32_t si = 0; si < S; si++) {
            const pg_leaf& pl = plan->segments[si].leaves[li];
            const LeafDesc& dl = leaves[(uint64_t)si * L + li];
            if ((dl.kind == LK_RANGE || dl.kind == LK_SET_LDS || dl.kind == LK_SET_LUT) &&
                (pl.kind != PG_LEAF_SV_SCAN || is_pre(li)))
              all_col = false;
          }
          if (all_col) q.leaf_slot[li] = (uint8_t)slot;
        }
      }
      if ((c.key >> 32) == 1 || (c.key >> 32) == 3) {
        const uint32_t cid = (uint32_t)c.key;
        const bool dec = (c.key >> 32) == 3;
        for (uint32_t a = 0; a < A; a++) {
          const pg_agg& g = plan->aggs[a];
          if (g.fn == PG_AGG_COUNT || g.fn == PG_AGG_COUNTMV || (g.flags & PG_AGG_MV_VALUES)) continue;
          if (g.col_a == cid && agg_dec(a, 0) == dec) q.agg_slot[a][0] = (uint8_t)slot;
          if (g.op != PG_EXPR_COL && g.fn != PG_AGG_DISTINCTCOUNT && g.col_b == cid && agg_dec(a, 1) == dec)
            q.agg_slot[a][1] = (uint8_t)slot;
        }
        for (uint32_t k = 0; k < K; k++)
          if (!((q.mv_keys >> k) & 1u) && plan->keys[k].col_id == cid && key_dec(k) == dec) q.key_slot[k] = (uint8_t)slot;
        // a leaf-sourced slot that aggregation / key uses share is sourced from one of those uses: their column words
        // exist in every segment, while a segment whose form of the leaf reads no column (isAlwaysTrue: LK_ALL) would
        // copy nothing and leave the shared slot stale for the aggregation
        if (c.role == 0) {
          bool moved = false;
          for (uint32_t a = 0; a < A && !moved; a++)
            for (uint32_t k = 0; k < 2 && !moved; k++)
              if (q.agg_slot[a][k] == slot) { q.staged[slot] = {1u, a, k, q.staged[slot].lds_word_off}; moved = true; }
          for (uint32_t k = 0; k < K && !moved; k++)
            if (q.key_slot[k] == slot) { q.staged[slot] = {2u, k, 0u, q.staged[slot].lds_word_off}; moved = true; }
        }
      }
    }
    q.stage_lds_words = words;
  }
  // ---- compaction queue: when the staged children of a root AND (phase A) pass few docs, the rest of the filter
  // and the aggregation (phase B) run over an LDS queue of their survivors, a full block of docs at a time,
  // instead of over the few survivors of each tile
  q.opA_begin = 0;
  q.opA_end = q.num_ops;
  q.opA_type = GT_ROOT;
  q.opB_begin = q.opB_end = 0;
  q.queue_mode = 0;
  if (q.num_ops && q.num_staged) {
    uint32_t a0 = 0, a1 = 0, type = GT_ROOT, b0 = 0, b1 = 0;
    double pass_a = 1.0;
    if (q.ops[0] >= 0) {
      if (q.leaf_slot[q.ops[0]] != kNoSlot) { a0 = 0; a1 = 1; pass_a = leaf_pass[q.ops[0]]; }
    } else if (q.ops[0] == kOpAnd) {
      uint32_t i = 1;
      while (i + 1 < q.num_ops && q.ops[i] >= 0 && q.leaf_slot[q.ops[i]] != kNoSlot) pass_a *= leaf_pass[q.ops[i++]];
      if (i > 1) { a0 = 1; a1 = i; type = GT_AND; b0 = i; b1 = q.num_ops - 1; }
    }
    bool agg_staged = false;
    for (uint32_t a = 0; a < A; a++) agg_staged |= q.agg_slot[a][0] != kNoSlot || q.agg_slot[a][1] != kNoSlot;
    for (uint32_t k = 0; k < K; k++) agg_staged |= q.key_slot[k] != kNoSlot;
    const bool work_after = b1 > b0 || K > 0 || q.agg_reads;
    static const char* queue_env = getenv("PG_QUEUE");
    const bool want = queue_env ? atoi(queue_env) != 0 : pass_a <= 1.0 / 16;
    if (a1 > a0 && !agg_staged && work_after && want) {
      q.queue_mode = 1;
      q.opA_begin = a0;
      q.opA_end = a1;
      q.opA_type = type;
      q.opB_begin = b0;
      q.opB_end = b1;
      for (uint32_t i = b0; i < b1; i++)  // phase B reads queued docs by gather only
        if (q.ops[i] >= 0) q.leaf_slot[q.ops[i]] = kNoSlot;
    }
  }
  {
    // two staging buffers (the copy of the next tile overlaps the current one) only when LDS still allows as many
    // blocks per CU as the register budget does (PG_SCAN_MIN_WAVES); else one.  PG_STAGE_RING=1|2 overrides.
    static const char* ring_env = getenv("PG_STAGE_RING");
    q.stage_ring = 2;
    const bool fits = q.num_staged && scan_lds_bytes(q) * (size_t)scan_min_blocks_per_cu(K > 0) <= 160 * 1024;
    q.stage_ring = ring_env ? (atoi(ring_env) > 1 ? 2 : 1) : (fits ? 2 : 1);
  }
  PG_PROF("queue");
  // ---- selective stream (pg_filter.hip stream_kernel): when the root AND's first child (or the whole filter) is a
  // packed scan leaf that passes few docs, a lean kernel streams that one column at full HBM rate and compacts its
  // survivors; the scan kernel then runs in list mode over them (the rest of the AND + aggregation, gathers only).
  // The fused tile loop pays a fixed cost per 8 192-doc tile that a 0.1 %-selective filter cannot amortise.
  // Regions hold 4x the expected survivors (+ slack); an overflow reruns the query without the stream.
  // PG_STREAM=0 disables, PG_STREAM_MAXPASS sets the pass-fraction bound (default 1/32).
  struct StreamLaunch { uint32_t bits, blocks; uint64_t first_off; std::vector<uint32_t> first; };
  struct StreamPlan {
    bool on = false;
    uint32_t leaf = 0, cap = 0;
    bool interleave = false;      // items dealt round-robin to the blocks (PG_STREAM_ITEM_GROUPS)
    bool exact = false;           // exact mode: the driving IN leaf's exact LUT staged in LDS (1 024-thread blocks)
    std::vector<uint32_t> exact_nwords;  // [seg] LUT words
    uint32_t set_ints = 0;        // LDS IN-set words of the streamed leaves
    std::vector<uint32_t> extra;  // further AND children tested in the stream (runtime bit width)
    double drive_pass = 1.0;      // the driving leaf's estimated pass fraction
    bool extra_lds_free = false;  // the further children need no LDS (allowed beside the exact mode's LUT)
    std::vector<StreamLaunch> launches;
    // overlapped list scan: launches [0, split_launch) stream the items [0, split) (the first half of the segments);
    // their list scan runs on a second stream while the remaining launches stream the rest (0: no overlap)
    uint32_t split = 0, split_launch = 0;
  } sp;
  {
    static const char* st_env = getenv("PG_STREAM");
    static const double max_pass = getenv("PG_STREAM_MAXPASS") ? atof(getenv("PG_STREAM_MAXPASS")) : 1.0 / 32;
    int32_t li = -1;
    double pass = 1.0;
    if (q.num_ops && q.ops[0] >= 0) {
      li = q.ops[0];
      pass = leaf_pass[li];
    } else if (q.num_ops > 2 && q.ops[0] == kOpAnd && q.ops[1] >= 0) {
      // the AND's leading leaf children while the joint pass is above 1/64: the first one streamed at its bit width,
      // the others tested on its survivors (doc ranges, constants, packed columns incl. 1-bit doc bitmaps)
      li = q.ops[1];
      pass = leaf_pass[li];
      sp.drive_pass = pass;
      for (uint32_t i = 2; i + 1 < q.num_ops && pass > 1.0 / 64 && sp.extra.size() < (size_t)kMaxStreamExtra; i++) {
        const int32_t lx = q.ops[i];
        if (lx < 0) break;
        bool fits = true;
        for (uint32_t si = 0; si < S && fits; si++) {
          const uint32_t k = leaves[(uint64_t)si * L + lx].kind;
          fits = k == LK_ALL || k == LK_NONE || k == LK_DOCRANGE || k == LK_RANGE || k == LK_SET_LDS || k == LK_SET_LUT;
        }
        if (!fits) break;
        sp.extra.push_back((uint32_t)lx);
        pass *= leaf_pass[lx];
      }
      // a driving leaf that passes <= 1/64 alone (config 2's accountId IN: 0.1 %): the following AND children that need
      // no LDS (doc ranges, constants, packed ranges, global-LUT sets) are still tested in the stream, on its few
      // survivors by per-doc windows -- the list scan then gets the AND's survivors instead of re-reading those
      // columns for every survivor of the driving leaf.  PG_STREAM_EXACT_EXTRA=1 enables it; off by default: measured
      // even on config 2 (stream 0.441 -> 0.492 ms, list scan 0.098 -> 0.050 ms, r04: the survivors' window reads stall
      // the streaming waves as long as the list kernel's gathers take)
      const char* xe_env = getenv("PG_STREAM_EXACT_EXTRA");  // read per call (tests switch it)
      if (sp.extra.empty() && pass <= 1.0 / 64 && xe_env && atoi(xe_env) == 1) {
        for (uint32_t i = 2; i + 1 < q.num_ops && sp.extra.size() < (size_t)kMaxStreamExtra; i++) {
          const int32_t lx = q.ops[i];
          if (lx < 0) break;
          bool fits = true;
          for (uint32_t si = 0; si < S && fits; si++) {
            const uint32_t k = leaves[(uint64_t)si * L + lx].kind;
            fits = k == LK_ALL || k == LK_NONE || k == LK_DOCRANGE || k == LK_RANGE || k == LK_SET_LUT;
          }
          if (!fits) break;
          sp.extra.push_back((uint32_t)lx);
          sp.extra_lds_free = true;
          pass *= leaf_pass[lx];
        }
      }
    }
    bool ok = allow_stream && !(plan->flags & PG_PLAN_NO_STREAM) && !(st_env && atoi(st_env) == 0) && li >= 0 &&
              !part.on && pre_leaves.empty() && pass <= max_pass && total_docs < 0xFFFFFFF0ull;
    std::map<uint32_t, std::vector<uint32_t>> by_bits;  // bit width -> segments whose form of the leaf reads it
    uint64_t T = 0;
    std::vector<uint64_t> seg_groups(S, 0);
    for (uint32_t si = 0; si < S && ok; si++) {
      if (!seg_tiles[si]) continue;
      const LeafDesc& dl = leaves[(uint64_t)si * L + li];
      if (dl.kind == LK_NONE) continue;
      ok = (dl.kind == LK_RANGE || dl.kind == LK_SET_LDS || dl.kind == LK_SET_LUT) && dl.bits >= 1 && dl.bits <= 32;
      by_bits[dl.bits].push_back(si);
      seg_groups[si] = ((uint64_t)plan->segments[si].num_docs + 31) / 32;
      T += seg_groups[si];
    }
    if (ok && T) {
      // items: per bit width, the concatenated 32-doc groups of its segments cut into one equal range per stream
      // block (blocks in proportion to the groups), split at segment boundaries; one launch per bit width
      static const char* ig_env = getenv("PG_STREAM_ITEM_GROUPS");  // > 0: interleaved items of this many groups
      static const char* bpc_env = getenv("PG_STREAM_BLOCKS_PER_CU");
      const uint64_t item_groups = ig_env ? (uint64_t)std::max(0, atoi(ig_env)) : 0;
      // blocks per CU: 7 (one resident round at 7 waves/SIMD) without further leaves; with them 12 (two rounds of the
      // 6-wave kernel: shorter ranges balance the survivors' gathers better; config 3 stream 0.639 -> 0.622 ms)
      // exact mode (PG_STREAM_EXACT=0 disables): a coarse IN bitmap whose exact LUT fits 128 KiB of LDS is tested
      // exactly by 1 024-thread blocks, one per CU, instead of resolving the coarse bitmap's candidates by global reads
      static const char* ex_env = getenv("PG_STREAM_EXACT");
      sp.exact = (sp.extra.empty() || sp.extra_lds_free) && !(ex_env && atoi(ex_env) == 0);
      sp.exact_nwords.assign(S, 0);
      for (uint32_t si = 0; si < S && sp.exact; si++) {
        if (!seg_groups[si]) continue;
        const LeafDesc& dl = leaves[(uint64_t)si * L + li];
        const ColumnRes* c = col(si, plan->segments[si].leaves[li].col_id);
        sp.exact = dl.kind == LK_SET_LDS && dl.shift > 0 && !dl.excl && c && (c->card + 31) / 32 <= 32768u;  // shift > 0: its exact LUT exists
        if (sp.exact) sp.exact_nwords[si] = (c->card + 31) / 32;
      }
      const uint64_t per_cu = sp.exact ? 1 : bpc_env ? (uint64_t)std::max(1, atoi(bpc_env)) : (sp.extra.empty() ? 7 : 12);
      const uint64_t NB = std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)g_num_cus * per_cu, T / 64));
      items.clear();
      uint64_t max_groups = 0;
      sp.interleave = item_groups > 0;
      for (auto& bb : by_bits) {
        if (sp.interleave) {  // items of item_groups groups in segment order, dealt round-robin to the blocks
          StreamLaunch sl;
          sl.bits = bb.first;
          const uint32_t first = (uint32_t)items.size();
          for (uint32_t si : bb.second)
            for (uint64_t g0 = 0; g0 < seg_groups[si]; g0 += item_groups) {
              const uint64_t e = std::min(seg_groups[si], g0 + item_groups);
              items.push_back({si, (uint32_t)g0, (uint32_t)e, 0});
              max_groups = std::max(max_groups, e - g0);
            }
          const uint64_t n_it = items.size() - first;
          sl.blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_it, (NB * n_it + 1) / std::max<uint64_t>(1, T / item_groups)));
          sl.first.assign(sl.blocks + 1, 0);
          sl.first[0] = first;
          sl.first[sl.blocks] = (uint32_t)items.size();
          sp.launches.push_back(std::move(sl));
          continue;
        }
        // overlapped list scan (exact mode, one bit width, >= 2 segments, a shape that fits beside the stream):
        // two launches over the two halves of the segments, each on the whole chip.  PG_LIST_OVERLAP=1 enables it
        // (read per call); off by default: config 2 measured 0.714 vs 0.644 ms per query -- the two stream launches
        // took 0.514 ms instead of 0.445 (the first half's list scan, running beside the second launch, slows it by
        // as much as it saves)
        const char* ov_env = getenv("PG_LIST_OVERLAP");
        std::vector<std::vector<uint32_t>> parts;
        if (sp.exact && by_bits.size() == 1 && bb.second.size() >= 2 && scan_co_resident(q) && ov_env &&
            atoi(ov_env) == 1) {
          uint64_t acc = 0;
          size_t cut = 0;
          while (cut + 1 < bb.second.size() && 2 * (acc + seg_groups[bb.second[cut]]) <= T) acc += seg_groups[bb.second[cut++]];
          if (cut == 0) cut = 1;
          parts.emplace_back(bb.second.begin(), bb.second.begin() + cut);
          parts.emplace_back(bb.second.begin() + cut, bb.second.end());
        } else {
          parts.push_back(bb.second);
        }
        for (size_t pi = 0; pi < parts.size(); pi++) {
          const std::vector<uint32_t>& segs_b = parts[pi];
          uint64_t Tb = 0;
          for (uint32_t si : segs_b) Tb += seg_groups[si];
          const uint64_t nb = parts.size() > 1 ? std::max<uint64_t>(1, std::min<uint64_t>(Tb, NB))
                                               : std::max<uint64_t>(1, std::min<uint64_t>(Tb, (NB * Tb + T - 1) / T));
          StreamLaunch sl;
          sl.bits = bb.first;
          sl.blocks = (uint32_t)nb;
          sl.first.assign(nb + 1, 0);
          size_t k = 0;
          uint64_t seg_first = 0;
          // block b's groups [b Tb / nb, (b + 1) Tb / nb), stepped by quotient + remainder (no divisions)
          const uint64_t dq = Tb / nb, dr = Tb % nb;
          uint64_t t1 = 0, rem = 0;
          for (uint64_t b = 0; b < nb; b++) {
            sl.first[b] = (uint32_t)items.size();
            uint64_t t0 = t1;
            t1 += dq;
            rem += dr;
            if (rem >= nb) { t1++; rem -= nb; }
            while (t0 < t1) {
              while (t0 >= seg_first + seg_groups[segs_b[k]]) { seg_first += seg_groups[segs_b[k]]; k++; }
              const uint64_t e = std::min(t1, seg_first + seg_groups[segs_b[k]]);
              items.push_back({segs_b[k], (uint32_t)(t0 - seg_first), (uint32_t)(e - seg_first), 0});
              max_groups = std::max(max_groups, e - t0);
              t0 = e;
            }
          }
          sl.first[nb] = (uint32_t)items.size();
          sp.launches.push_back(std::move(sl));
          if (parts.size() > 1 && pi == 0) {
            sp.split = (uint32_t)items.size();
            sp.split_launch = (uint32_t)sp.launches.size();
          }
        }
      }
      const double expect = pass * 32.0 * (double)max_groups;
      const uint64_t slack = std::min<uint64_t>(1024, std::max<uint64_t>(64, 8 * max_groups));
      const uint64_t cap = std::min<uint64_t>(32 * max_groups, ((uint64_t)(4.0 * expect) + slack + 63) & ~63ull);
      sp.on = true;
      sp.leaf = (uint32_t)li;
      sp.cap = (uint32_t)cap;
      q.num_items = (uint32_t)items.size();
      static const char* lb_env = getenv("PG_LIST_BLOCKS");
      // list grid: ~2 048 expected survivors per block, 256..4 x CUs blocks (fewer blocks = fewer flushes of the block
      // group tables; measured: config 2 (1 M survivors) 512 blocks 0.099 ms vs 1 536 0.166 ms; config 3 (14 M)
      // 768-1 024 blocks 0.297 ms vs 1 536 0.333 ms: tools/stream_sweep*.sh)
      const uint64_t want = std::max<uint64_t>(256, (uint64_t)(pass * 32.0 * (double)T) / 2048);
      grid = (uint32_t)std::min<uint64_t>(items.size(), lb_env ? (uint64_t)std::max(1, atoi(lb_env))
                                                                : std::min<uint64_t>(want, (uint64_t)g_num_cus * 4));
      want_xcd = false;
      // list mode: the driving leaf is done; phase B = the AND's remaining children, all read by gathers
      q.list_mode = 1;
      q.list_cap = sp.cap;
      q.queue_mode = 1;
      q.opA_begin = q.opA_end = 0;
      q.opA_type = GT_ROOT;
      if (q.ops[0] >= 0) { q.opB_begin = q.opB_end = 0; }
      else { q.opB_begin = 2 + (uint32_t)sp.extra.size(); q.opB_end = q.num_ops - 1; }
      q.num_staged = 0;
      q.stage_lds_words = 0;
      q.stage_ring = 1;
      memset(q.leaf_slot, kNoSlot, sizeof(q.leaf_slot));
      memset(q.agg_slot, kNoSlot, sizeof(q.agg_slot));
      memset(q.key_slot, kNoSlot, sizeof(q.key_slot));
      // the list kernel stages only the IN sets its phase-B leaves read (the streamed leaves' sets are the stream's)
      sp.set_ints = q.set_lds_ints;
      bool b_sets = false;
      for (uint32_t i = q.opB_begin; i < q.opB_end; i++)
        for (uint32_t si = 0; si < S && q.ops[i] >= 0 && !b_sets; si++)
          b_sets = leaves[(uint64_t)si * L + q.ops[i]].kind == LK_SET_LDS;
      if (!b_sets) q.set_lds_ints = 0;
    }
  }
  const size_t lds_bytes = scan_lds_bytes(q);
  if (lds_bytes > 160 * 1024) return fail(PG_E_UNSUPPORTED, "scan needs %zu bytes of LDS", lds_bytes);

  PG_PROF("stream");
  // ---- fused index count (pg_index.hip): COUNT / COUNTMV with no group-by under a filter of index leaves only
  // (inverted dictId sets, sorted doc ranges, constants) in at most two levels of AND / OR / NOT: one launch decodes
  // each 64 K-doc key's containers into LDS, evaluates the filter there and counts -- instead of the roaring pre-pass
  // writing doc bitmaps to HBM and the fused scan reading them back.  PG_INDEX_FUSED=0 disables.
  struct IdxPlan {
    bool on = false;
    IdxSpec spec{};
    std::vector<IdxLeaf> leaves;        // [S][L]
    std::vector<IdxSeg> segs;           // [S]
    std::vector<uint64_t> ids_off;      // [S][L] arena offset of a ROARING leaf's dictIds (~0: none)
    uint32_t blocks = 0;
  } ix;
  {
    const char* ix_env = getenv("PG_INDEX_FUSED");
    bool ok = !(ix_env && atoi(ix_env) == 0) && K == 0 && A >= 1 && L <= kIdxMaxLeaves && !part.on && !sp.on &&
              pre_leaves.empty() && luts.empty();  // the scratch (LUTs, bitmaps) is not allocated when fused
    uint32_t cntmv = 0xFFFFFFFFu, cntmv_col = 0;
    for (uint32_t a = 0; a < A && ok; a++) {
      const pg_agg& g = plan->aggs[a];
      if (g.fn == PG_AGG_COUNT) continue;
      ok = g.fn == PG_AGG_COUNTMV && cntmv == 0xFFFFFFFFu;
      cntmv = P.aggs[a].slot;
      cntmv_col = g.col_a;
    }
    std::vector<int> roar((uint64_t)S * L, -1);  // (segment, leaf) -> its ROARING pre-pass op
    for (size_t k = 0; k < pre.size() && ok; k++) {
      ok = pre[k].kind == PrepassOp::ROARING;
      if (ok) roar[(uint64_t)pre[k].seg * L + pre[k].leaf] = (int)k;
    }
    // the filter as items of a root AND / OR, each a leaf or a group (AND / OR of leaves), any of them negated
    IdxSpec& sp2 = ix.spec;
    if (ok && plan->num_ops) {
      struct N { int kind, leaf; std::vector<int> kids; };  // 0 leaf, 1 AND, 2 OR, 3 NOT
      std::vector<N> nodes;
      std::vector<int> st;
      for (uint32_t i = 0; i < plan->num_ops; i++) {
        const int32_t op = plan->ops[i];
        N n{0, -1, {}};
        if (op >= 0) { n.leaf = op; }
        else {
          const int cnt = op == PG_OP_NOT ? 1 : ((-op) & 0xFF);
          n.kind = op == PG_OP_NOT ? 3 : (((-op) & 0x300) == 0x100 ? 1 : 2);
          n.kids.assign(st.end() - cnt, st.end());
          st.resize(st.size() - cnt);
        }
        nodes.push_back(n);
        st.push_back((int)nodes.size() - 1);
      }
      uint32_t ng = 0, ngl = 0;
      // a leaf or NOT leaf -> gleaf / item code; -1 if not a (negated) leaf
      auto leaf_code = [&](int x) -> int64_t {
        bool neg = false;
        while (nodes[x].kind == 3) { neg = !neg; x = nodes[x].kids[0]; }
        if (nodes[x].kind != 0) return -1;
        return (int64_t)((uint32_t)nodes[x].leaf | (neg ? 0x80000000u : 0u));
      };
      auto item_code = [&](int x) -> int64_t {
        const int64_t lc = leaf_code(x);
        if (lc >= 0) return lc;
        bool neg = false;
        while (nodes[x].kind == 3) { neg = !neg; x = nodes[x].kids[0]; }
        if (ng >= kIdxMaxItems) return -1;
        const uint32_t g = ng++;
        sp2.group_or[g] = nodes[x].kind == 2;
        sp2.gfirst[g] = ngl;
        sp2.gn[g] = (uint32_t)nodes[x].kids.size();
        for (int k : nodes[x].kids) {
          const int64_t c = leaf_code(k);
          if (c < 0 || ngl >= kIdxMaxItems) return -1;
          sp2.gleaf[ngl++] = (uint32_t)c;
        }
        return (int64_t)(g | 0x40000000u | (neg ? 0x80000000u : 0u));
      };
      const int root = st.back();
      std::vector<int> items1;
      if (nodes[root].kind == 1 || nodes[root].kind == 2) { sp2.root_or = nodes[root].kind == 2; items1 = nodes[root].kids; }
      else { sp2.root_or = 0; items1.push_back(root); }
      ok = items1.size() <= kIdxMaxItems;
      for (size_t i = 0; i < items1.size() && ok; i++) {
        const int64_t c = item_code(items1[i]);
        ok = c >= 0;
        if (ok) sp2.item[sp2.num_items++] = (uint32_t)c;
      }
    } else if (ok) {
      sp2.root_or = 0;  // no filter: every doc
      sp2.num_items = 0;
    }
    // the leaves of each segment: constants, doc ranges, inverted leaves (their LDS chunk slots)
    if (ok) {
      for (uint32_t l = 0; l < kIdxMaxLeaves; l++) sp2.chunk_of[l] = 0xFFFFFFFFu;
      ix.leaves.assign((uint64_t)S * L, IdxLeaf{});
      ix.ids_off.assign((uint64_t)S * L, ~0ull);
      ix.segs.assign(S, IdxSeg{});
      for (uint32_t si = 0; si < S && ok; si++) {
        for (uint32_t li = 0; li < L && ok; li++) {
          const LeafDesc& dl = leaves[(uint64_t)si * L + li];
          IdxLeaf& x = ix.leaves[(uint64_t)si * L + li];
          const int r = roar[(uint64_t)si * L + li];
          if (r >= 0) {
            const PrepassOp& op = pre[r];
            x.kind = IL_ROARING;
            x.negate = op.negate ? 1u : 0u;
            x.roaring = (const uint8_t*)op.col->roaring.p;
            x.cs = (const RoaringContainer*)op.col->containers.p;
            x.dir = (const uint32_t*)op.col->inv_dir_dev.p;
            x.keydir = (const uint2*)op.col->inv_keydir.p;
            x.card = op.col->inv_keydir_card;
            x.nids = op.n;
            ix.ids_off[(uint64_t)si * L + li] = op.in_off;
            if (sp2.chunk_of[li] == 0xFFFFFFFFu) sp2.chunk_of[li] = sp2.num_chunks++;
          } else if (dl.kind == LK_ALL) { x.kind = IL_ALL; }
          else if (dl.kind == LK_NONE) { x.kind = IL_NONE; }
          else if (dl.kind == LK_DOCRANGE) { x.kind = IL_DOCRANGE; x.lo = dl.lo; x.hi = dl.hi; }
          else ok = false;
        }
        IdxSeg& g = ix.segs[si];
        g.num_docs = plan->segments[si].num_docs;
        const uint32_t lo = root_range[si].first, hi = std::min(root_range[si].second, g.num_docs);
        const uint32_t nk = (nonscan[si] || !seg_tiles[si] || hi <= lo) ? 0u : ((hi - 1) >> 16) + 1 - (lo >> 16);
        g.key0 = nk ? lo >> 16 : 0u;
        g.first_block = ix.blocks;
        ix.blocks += nk;
        if (ok && cntmv != 0xFFFFFFFFu && nk) {  // (ok: a leaf above may have ruled the fused count out)
          const ColumnRes* c = col(si, cntmv_col);
          ok = c && c->fwd == FWD_MV && c->mv_offsets.p;
          if (ok) {
            g.mv_cnt = (const uint32_t*)c->mv_cnt.p;
            g.mv_offsets = (const uint32_t*)c->mv_offsets.p;
          }
        }
      }
    }
    if (ok && sp2.num_chunks > 1) {
      // the positive inverted leaves of one OR (a group, or the root's leaf items) decode into ONE chunk: the OR of
      // their containers is the union either of them then reads (a constant or doc-range form in some segment still
      // ORs in correctly) -- fewer LDS chunks per block, more blocks per CU
      bool neg[kIdxMaxLeaves] = {};
      for (uint64_t k = 0; k < ix.leaves.size(); k++)
        if (ix.leaves[k].kind == IL_ROARING && ix.leaves[k].negate) neg[k % L] = true;
      // only a leaf the program references ONCE may read the OR's union: `a AND (a OR c)` references leaf a twice,
      // and its AND must see a's own docs
      uint32_t refs[kIdxMaxLeaves] = {};
      for (uint32_t i = 0; i < plan->num_ops; i++)
        if (plan->ops[i] >= 0 && (uint32_t)plan->ops[i] < kIdxMaxLeaves) refs[plan->ops[i]]++;
      uint32_t rep[kIdxMaxLeaves];
      for (uint32_t l = 0; l < kIdxMaxLeaves; l++) rep[l] = l;
      auto share = [&](const uint32_t* codes, uint32_t n) {
        int first = -1;
        for (uint32_t k = 0; k < n; k++) {
          const uint32_t c = codes[k];
          if (c & 0xC0000000u) continue;  // a group or a negated item
          const uint32_t l = c & 0xFFu;
          if (l >= L || neg[l] || refs[l] != 1 || sp2.chunk_of[l] == 0xFFFFFFFFu) continue;
          if (first < 0) first = (int)l; else rep[l] = (uint32_t)first;
        }
      };
      for (uint32_t gi = 0; gi < kIdxMaxItems; gi++)
        if (sp2.group_or[gi] && sp2.gn[gi]) share(sp2.gleaf + sp2.gfirst[gi], sp2.gn[gi]);
      if (sp2.root_or) share(sp2.item, sp2.num_items);
      uint32_t newc[kIdxMaxLeaves];
      for (uint32_t l = 0; l < kIdxMaxLeaves; l++) newc[l] = 0xFFFFFFFFu;
      sp2.num_chunks = 0;
      for (uint32_t l = 0; l < L; l++) {
        if (sp2.chunk_of[l] == 0xFFFFFFFFu) continue;
        if (newc[rep[l]] == 0xFFFFFFFFu) newc[rep[l]] = sp2.num_chunks++;
        sp2.chunk_of[l] = newc[rep[l]];
      }
    }
    if (ok) {
      ix.on = true;
      sp2.num_segs = S;
      sp2.num_leaves = L;
      sp2.cntmv_slot = cntmv;
      q.num_items = 0;          // no fused scan
      items.clear();
      scratch_bytes = 0;        // nor doc bitmaps: the scratch would only hold the unused ones
    }
  }
  // ---- device buffers (state + arena + scratch) from the caching pool
  part.on = part.on && q.num_items > 0;
  // the state's byte fills ride on the arena-upload launch unless the non-scan seeding below writes the state first
  FillSpans fills;
  memset(&fills, 0, sizeof(fills));
  const bool defer_fills = !(ns_docs || ns_matched);
  if ((rc = P.alloc_state(s, !part.on, defer_fills ? &fills : nullptr))) return rc;
  if (ns_docs || ns_matched) {  // the non-scan segments' results seed the state the scan adds to
    uint64_t* h = (uint64_t*)t_ctx.readback.get(8ull * (1 + 2 * A));
    if (!h) return fail(PG_E_NOMEM, "pinned staging failed");
    h[0] = ns_docs;
    HIP_CHECK(hipMemcpyAsync(P.i64.p, &h[0], 8, hipMemcpyHostToDevice, s));
    for (uint32_t a = 0; a < A; a++) {
      const pg_agg& g = plan->aggs[a];
      if (g.fn != PG_AGG_MIN && g.fn != PG_AGG_MAX) continue;
      double m = g.fn == PG_AGG_MIN ? INFINITY : -INFINITY;
      for (uint32_t si = 0; si < S; si++) {
        if (!nonscan[si]) continue;
        const ColumnRes* c = col(si, g.col_a);
        if (c->card || c->fwd == FWD_RAW) m = g.fn == PG_AGG_MIN ? std::min(m, c->dmin) : std::max(m, c->dmax);
      }
      h[1 + a] = (uint64_t)order_key(m);
      void* dst = g.fn == PG_AGG_MIN ? (void*)((long long*)P.mn.p + P.aggs[a].slot) : (void*)((long long*)P.mx.p + P.aggs[a].slot);
      HIP_CHECK(hipMemcpyAsync(dst, &h[1 + a], 8, hipMemcpyHostToDevice, s));
    }
    for (uint32_t a = 0; a < A; a++) {
      const pg_agg& g = plan->aggs[a];
      if (g.fn != PG_AGG_DISTINCTCOUNT) continue;
      for (uint32_t si = 0; si < S; si++) {
        if (!nonscan[si]) continue;
        const ColumnRes* c = col(si, g.col_a);
        HIP_CHECK(launch_dict_bits(c->dict.p, c->dtype, c->card, g.key_base,
                                   g.key_kind == PG_KEY_KEYMAP ? (const int32_t*)c->keymap.p : nullptr, g.key_cardinality,
                                   (uint32_t*)P.bits.p + P.aggs[a].dc_word, (unsigned int*)P.misc.p + 1, s));
      }
    }
    HIP_CHECK(hipStreamSynchronize(s));  // the pinned staging words are reused below
  }
  // [S] matched docs | error word | pad | the stream's two wall-clock stamps (StreamSpec.stamp): read back together
  if ((rc = P.seg_matched.alloc_pooled(8ull * (S ? S : 1) + 32))) return rc;
  if (!fills.add(P.seg_matched.p, 0, 8ull * (S ? S : 1) + 32))
    HIP_CHECK(hipMemsetAsync(P.seg_matched.p, 0, 8ull * (S ? S : 1) + 32, s));
  {
    const StateView v = P.view();
    q.i64 = v.i64;
    q.fx = v.fx;
    q.mn = v.mn;
    q.mx = v.mx;
    q.dbits = v.bits;
    q.hkeys = v.keys;
    q.hfill = v.fill;
    q.first_doc = v.first_doc;
  }
  q.seg_matched = (unsigned long long*)P.seg_matched.p;
  q.err = (unsigned int*)(q.seg_matched + (S ? S : 1));

  const uint64_t off_leaves = ar.reserve(leaves.size() * sizeof(LeafDesc));
  const uint64_t off_aggcols = ar.reserve(aggcols.size() * sizeof(ColDesc));
  const uint64_t off_keycols = ar.reserve(keycols.size() * sizeof(ColDesc));
  const uint64_t off_segs = ar.reserve(segd.size() * sizeof(SegDesc));
  // the pre-filter's view: the original (unfolded) leaves, their segment table, its output bitmaps
  const uint64_t off_leaves_orig = ar.reserve(leaves_orig.size() * sizeof(LeafDesc));
  const uint64_t off_segs_pre = ar.reserve(pre_leaves.empty() ? 0 : segd.size() * sizeof(SegDesc));
  const uint64_t off_pre_out = ar.reserve(pre_leaves.empty() ? 0 : 8ull * S);
  uint32_t blocks = 0;
  if (!items.empty()) {
    blocks = grid;
    // XCD-grouped item order when the query decodes a large dictionary for many docs (> 16 decodes per
    // 128-byte dictionary line per segment; SSB SUM(lo_extendedprice) over all rows: 13.2 -> 4.7 ms): workgroups are dispatched round-robin over the 8 XCDs (block b ->
    // XCD b % 8), each with its own L2.  Give each XCD a contiguous run of segments and, within it, interleave
    // the items step-major over the XCD's blocks, so at any moment the blocks of one XCD scan the same segment
    // and share its dictionary lines in their L2 (instead of every XCD pulling every dictionary).
    constexpr uint32_t kXcds = 8;
    if (want_xcd && blocks % kXcds == 0 && blocks >= 2 * kXcds) {
      const uint64_t N = items.size();
      std::vector<WorkItem>& out = t_ctx.items_perm;
      out.resize(N);
      auto range_len = [&](uint32_t b) { return (uint32_t)(((uint64_t)b + 1) * N / blocks - (uint64_t)b * N / blocks); };
      uint64_t next = 0;  // next item (segment order) to hand out
      for (uint32_t x = 0; x < kXcds; x++) {
        uint32_t max_r = 0;
        for (uint32_t b = x; b < blocks; b += kXcds) max_r = std::max(max_r, range_len(b));
        for (uint32_t j = 0; j < max_r; j++)
          for (uint32_t b = x; b < blocks; b += kXcds)
            if (j < range_len(b)) out[(uint64_t)b * N / blocks + j] = items[next++];
      }
      items.swap(out);
    }
  }
  const uint64_t off_items = ar.put(items.data(), items.size() * sizeof(WorkItem));
  for (StreamLaunch& sl : sp.launches) sl.first_off = ar.put(sl.first.data(), sl.first.size() * 4);
  // exact-mode segments whose driving leaf's LUT the stream builds in LDS (ids mode; the leaf read nowhere else: not a
  // further stream leaf, not in the list scan's phase B); PG_STREAM_LDS_LUT=0 keeps the global LUT staging
  std::vector<uint8_t> lds_lut(S, 0);
  std::vector<size_t> exact_req(S, 0);  // the LutReq (ids or literals) of segment si's driving leaf
  std::vector<LutReq> exact_luts;
  {
    const char* ll_env = getenv("PG_STREAM_LDS_LUT");
    bool ok = sp.on && sp.exact && q.num_items && !(ll_env && atoi(ll_env) == 0);
    for (uint32_t x : sp.extra) ok = ok && x != sp.leaf;
    for (uint32_t i = q.opB_begin; i < q.opB_end && ok; i++) ok = q.ops[i] != (int32_t)sp.leaf;
    if (ok)
      for (const SetLdsRes& x : set_lds_res) {
        const uint32_t si = (uint32_t)(x.leaf_index / L), li = (uint32_t)(x.leaf_index % L);
        if (li != sp.leaf || !sp.exact_nwords[si]) continue;
        lds_lut[si] = 1;
        exact_req[si] = exact_luts.size();
        exact_luts.push_back(luts[x.lut_req]);
      }
    std::vector<uint8_t> drop(luts.size(), 0);
    for (const SetLdsRes& x : set_lds_res) {
      const uint32_t si = (uint32_t)(x.leaf_index / L), li = (uint32_t)(x.leaf_index % L);
      if (lds_lut[si] && li == sp.leaf) {
        drop[x.lut_req] = 1;
        continue;
      }
      LutReq& lr = luts[x.lut_req];
      lr.region_off = scratch_reserve(x.region_bytes);
      patches.push_back({x.leaf_index, lr.region_off, false, PT_AUX});
      if (x.lut_bytes) {
        lr.lut_off = scratch_reserve(x.lut_bytes);
        patches.push_back({x.leaf_index, lr.lut_off, false, PT_LUT});
      }
    }
    size_t k = 0;
    for (size_t i = 0; i < luts.size(); i++)
      if (!drop[i]) luts[k++] = luts[i];
    luts.resize(k);
  }
  const uint64_t off_exact = sp.exact ? ar.reserve(S * sizeof(ExactSet)) : 0;
  // GM_PART: each block's region of the entry array = the docs of its items (the kernel's [i0, i1) item range)
  uint64_t off_part_base = 0, part_entries = 0;
  if (part.on && blocks) {
    std::vector<uint64_t> base(blocks + 1, 0);
    for (uint32_t b = 0; b < blocks; b++) {
      const uint64_t i0 = (uint64_t)b * items.size() / blocks, i1 = (uint64_t)(b + 1) * items.size() / blocks;
      uint64_t n = 0;
      for (uint64_t i = i0; i < i1; i++) {
        const WorkItem& it = items[i];
        const uint64_t nd = plan->segments[it.seg].num_docs;
        n += std::min<uint64_t>((uint64_t)it.tile_end * kTileDocs, nd) - std::min<uint64_t>((uint64_t)it.tile_begin * kTileDocs, nd);
      }
      base[b + 1] = base[b] + n;
    }
    part_entries = base[blocks];
    off_part_base = ar.put(base.data(), base.size() * 8);
  }
  const uint64_t off_lutjobs = ar.reserve(luts.size() * sizeof(LutJob));
  std::vector<RoaringJob> rjobs;
  uint32_t roaring_blocks = 0;
  for (const PrepassOp& op : pre) {
    if (ix.on || op.kind != PrepassOp::ROARING || !op.nkeys) continue;
    RoaringJob j;
    memset(&j, 0, sizeof(j));
    j.nids = op.n;
    j.num_docs = op.num_docs;
    j.negate = op.negate ? 1u : 0u;
    j.key0 = op.key0;
    j.nkeys = op.nkeys;
    j.first_block = roaring_blocks;
    roaring_blocks += op.nkeys;
    rjobs.push_back(j);
  }
  const uint64_t off_rjobs = ar.reserve(rjobs.size() * sizeof(RoaringJob));
  const uint64_t off_ixleaves = ar.reserve(ix.leaves.size() * sizeof(IdxLeaf));
  const uint64_t off_ixsegs = ar.reserve(ix.segs.size() * sizeof(IdxSeg));
  const uint64_t off_ixblk = ar.reserve(ix.on ? 4ull * ix.blocks : 0ull);  // block -> segment
  DevBuf arena, scratch;
  DevBuf p_ent0, p_cnt0, p_hist1, p_off1, p_ent1, p_hist2, p_off2, p_ent2, p_temp, p_fill;  // GM_PART pipeline
  DevBuf l_docs, l_counts;  // selective stream: survivor regions + counts
  // declared after the buffers it protects: on any exit, wait for queued work before they return to the pool
  struct SyncOnExit {
    hipStream_t s;
    bool s2 = false;  // an overlapped list-scan half was launched on the second stream
    ~SyncOnExit() {
      if (s2) (void)hipStreamSynchronize(t_ctx.s2);
      (void)hipStreamSynchronize(s);
    }
  } sync_on_exit{s};
  if ((rc = arena.alloc_pooled(ar.h.size() + 16))) return rc;
  if (scratch_bytes && (rc = scratch.alloc_pooled(scratch_bytes))) return rc;
  uint8_t* dA = (uint8_t*)arena.p;
  uint8_t* dS = (uint8_t*)scratch.p;
  for (const Patch& p : patches) {
    LeafDesc& dl = (p.orig ? leaves_orig : leaves)[p.leaf_index];
    const uint32_t* ptr = (const uint32_t*)((p.in_arena ? dA : dS) + p.off);
    if (p.target == PT_WORDS) dl.words = ptr;
    else if (p.target == PT_LUT) dl.lut = ptr;
    else if (p.target == PT_RVALS) dl.rvals = ptr;
    else dl.aux = ptr;
  }
  for (uint32_t si = 0; si < S; si++) {
    segd[si].leaves = (const LeafDesc*)(dA + off_leaves) + (uint64_t)si * L;
    segd[si].aggcols = (const ColDesc*)(dA + off_aggcols) + (uint64_t)si * A * 2;
    segd[si].keycols = (const ColDesc*)(dA + off_keycols) + (uint64_t)si * K;
  }
  std::vector<LutJob> lutjobs(luts.size());
  for (size_t i = 0; i < luts.size(); i++)
    lutjobs[i] = {luts[i].ids_off == ~0ull ? nullptr : (const int32_t*)(dA + luts[i].ids_off),
                  luts[i].lut_off == ~0ull ? nullptr : (uint32_t*)(dS + luts[i].lut_off),
                  luts[i].region_off == ~0ull ? nullptr : (uint32_t*)(dS + luts[i].region_off), luts[i].n, luts[i].shift,
                  luts[i].vals_off == ~0ull ? nullptr : (const void*)(dA + luts[i].vals_off), luts[i].dict,
                  luts[i].card, luts[i].dtype};
  if (!leaves.empty()) memcpy(&ar.h[off_leaves], leaves.data(), leaves.size() * sizeof(LeafDesc));
  if (!aggcols.empty()) memcpy(&ar.h[off_aggcols], aggcols.data(), aggcols.size() * sizeof(ColDesc));
  if (!keycols.empty()) memcpy(&ar.h[off_keycols], keycols.data(), keycols.size() * sizeof(ColDesc));
  if (!segd.empty()) memcpy(&ar.h[off_segs], segd.data(), segd.size() * sizeof(SegDesc));
  if (!lutjobs.empty()) memcpy(&ar.h[off_lutjobs], lutjobs.data(), lutjobs.size() * sizeof(LutJob));
  if (sp.exact) {
    std::vector<ExactSet> es(S);
    for (uint32_t si = 0; si < S; si++) {
      memset(&es[si], 0, sizeof(ExactSet));
      es[si].nwords = sp.exact_nwords[si];
      if (!lds_lut[si]) continue;
      const LutReq& x = exact_luts[exact_req[si]];
      es[si].n = x.n;
      if (x.ids_off != ~0ull) {
        es[si].ids = (const int32_t*)(dA + x.ids_off);
      } else {  // values mode: the literals (dictionary's stored type) and the segment's dictionary
        es[si].vals = dA + x.vals_off;
        es[si].dict = x.dict;
        es[si].card = x.card;
        es[si].dtype = x.dtype;
      }
    }
    memcpy(&ar.h[off_exact], es.data(), S * sizeof(ExactSet));
  }
  {
    size_t k = 0;
    for (const PrepassOp& op : pre) {
      if (ix.on || op.kind != PrepassOp::ROARING || !op.nkeys) continue;  // the same selection as the job list above
      RoaringJob& j = rjobs[k++];
      j.roaring = (const uint8_t*)op.col->roaring.p;
      j.cs = (const RoaringContainer*)op.col->containers.p;
      j.dir = (const uint32_t*)op.col->inv_dir_dev.p;
      j.keydir = (const uint2*)op.col->inv_keydir.p;
      j.card = op.col->inv_keydir_card;
      j.ids = (const int32_t*)(dA + op.in_off);
      j.bm = (uint32_t*)(dS + op.out_off);
    }
    if (!rjobs.empty()) memcpy(&ar.h[off_rjobs], rjobs.data(), rjobs.size() * sizeof(RoaringJob));
  }
  if (ix.on) {  // the fused index count's leaf / segment tables (dictId lists already in the arena)
    for (size_t k = 0; k < ix.leaves.size(); k++)
      if (ix.ids_off[k] != ~0ull) ix.leaves[k].ids = (const int32_t*)(dA + ix.ids_off[k]);
    for (uint32_t si = 0; si < S; si++) ix.segs[si].leaves = (const IdxLeaf*)(dA + off_ixleaves) + (uint64_t)si * L;
    if (!ix.leaves.empty()) memcpy(&ar.h[off_ixleaves], ix.leaves.data(), ix.leaves.size() * sizeof(IdxLeaf));
    if (!ix.segs.empty()) memcpy(&ar.h[off_ixsegs], ix.segs.data(), ix.segs.size() * sizeof(IdxSeg));
    ix.spec.segs = (const IdxSeg*)(dA + off_ixsegs);
    ix.spec.leaves = (const IdxLeaf*)(dA + off_ixleaves);
    uint32_t* bs = (uint32_t*)&ar.h[off_ixblk];
    for (uint32_t si = 0; si < S; si++)
      for (uint32_t b = ix.segs[si].first_block; b < (si + 1 < S ? ix.segs[si + 1].first_block : ix.blocks); b++) bs[b] = si;
    ix.spec.blk_seg = (const uint32_t*)(dA + off_ixblk);
    ix.spec.i64 = (unsigned long long*)P.i64.p;
    ix.spec.seg_matched = (unsigned long long*)P.seg_matched.p;
  }
  if (!pre_leaves.empty()) {
    memcpy(&ar.h[off_leaves_orig], leaves_orig.data(), leaves_orig.size() * sizeof(LeafDesc));
    std::vector<SegDesc> segp(segd);
    std::vector<uint32_t*> outs(S);
    for (uint32_t si = 0; si < S; si++) {
      segp[si].leaves = (const LeafDesc*)(dA + off_leaves_orig) + (uint64_t)si * L;
      outs[si] = (uint32_t*)(dS + pre_bitmap_off[si]);
    }
    memcpy(&ar.h[off_segs_pre], segp.data(), segp.size() * sizeof(SegDesc));
    memcpy(&ar.h[off_pre_out], outs.data(), outs.size() * 8);
  }
  q.segs = (const SegDesc*)(dA + off_segs);
  q.items = (const WorkItem*)(dA + off_items);

  hipEvent_t* ev = t_ctx.ev;
  PG_PROF("arena");
  // the arena was built in pinned memory: the device reads it from there
  HIP_CHECK(launch_arena_upload(ar.h.dp, arena.p, ar.h.size(), scratch.p, scratch_bytes, fills, s));
  HIP_CHECK(timing_record(ev[0], s));
  {
    uint32_t max_n = 0;
    for (const LutReq& r : luts) max_n = std::max(max_n, r.n);
    HIP_CHECK(launch_set_lut_bits((const LutJob*)(dA + off_lutjobs), (uint32_t)lutjobs.size(), max_n, s));
  }
  for (const PrepassOp& op : pre) {
    switch (op.kind) {
      case PrepassOp::FILL_RANGES:
        HIP_CHECK(launch_fill_ranges((const int32_t*)(dA + op.in_off), op.n, op.num_docs, (uint32_t*)(dS + op.out_off), s));
        break;
      case PrepassOp::ROARING:  // all of them in one launch below
        break;
      case PrepassOp::MV_SCAN:
        HIP_CHECK(launch_mv_scan((const uint32_t*)op.col->words.p, op.col->bits, (const uint32_t*)op.col->mv_offsets.p,
                                 op.num_docs, op.lo, op.hi,
                                 op.lut_off == ~0ull ? nullptr : (const uint32_t*)(dS + op.lut_off), op.excl,
                                 (uint32_t*)(dS + op.out_off), s));
        break;
    }
  }
  HIP_CHECK(launch_roaring_keys((const RoaringJob*)(dA + off_rjobs), (uint32_t)rjobs.size(), roaring_blocks, s));
  // the pre-pass's end, recorded only when a pre-pass kernel ran (an event record costs the stream a few us between
  // its dependent kernels: none was launched -> the pre-pass took no time and ev[0] stands for its end)
  const bool pre_ran = !lutjobs.empty() || !pre.empty() || (!rjobs.empty() && roaring_blocks);
  if (pre_ran) HIP_CHECK(timing_record(ev[4], s));
  hipEvent_t ev_pre = pre_ran ? ev[4] : ev[0];
  for (const PreLaunch& pl : pre_launches) {
    PreSpec ps;
    memset(&ps, 0, sizeof(ps));
    ps.num_items = pl.n_items;
    ps.leaf = pl.leaf;
    ps.first = pl.first;
    ps.set_lds_ints = pl.set_ints;
    ps.segs = (const SegDesc*)(dA + off_segs_pre);
    ps.items = (const WorkItem*)(dA + pl.items_off);
    ps.out = (uint32_t* const*)(dA + off_pre_out);
    HIP_CHECK(launch_prefilter(ps, pl.bits, (uint32_t)std::min<uint64_t>(pl.n_items, (uint64_t)g_num_cus * 8), s));
  }
  // the pre-filter kernels' end (the stream's own time comes from its stamps: no record between it and the scan)
  if (!pre_launches.empty()) HIP_CHECK(timing_record(ev[1], s));
  if (sp.on && q.num_items) {
    if ((rc = l_docs.alloc_pooled(4ull * q.num_items * sp.cap + 16)) || (rc = l_counts.alloc_pooled(4ull * q.num_items + 16)))
      return rc;
    StreamSpec ss;
    memset(&ss, 0, sizeof(ss));
    ss.num_items = q.num_items;
    ss.leaf = sp.leaf;
    ss.cap = sp.cap;
    ss.num_extra = (uint32_t)sp.extra.size();
    ss.exact = sp.exact ? (const ExactSet*)(dA + off_exact) : nullptr;
    ss.interleave = sp.interleave ? 1u : 0u;
    for (size_t x = 0; x < sp.extra.size(); x++) ss.extra[x] = sp.extra[x];
    ss.set_lds_ints = (sp.set_ints + 3u) & ~3u;  // the wave slices start 16-byte aligned after the IN sets
    {
      // wave slices for the further leaves' columns of <= kStreamStageBits bits (PG_STREAM_STAGE=0: per-doc windows)
      static const char* stg_env = getenv("PG_STREAM_STAGE");
      uint32_t bmax = 0;
      for (uint32_t x : sp.extra)
        for (uint32_t si = 0; si < S; si++) {
          const LeafDesc& dl = leaves[(uint64_t)si * L + x];
          if ((dl.kind == LK_RANGE || dl.kind == LK_SET_LDS || dl.kind == LK_SET_LUT) && dl.bits <= kStreamStageBits)
            bmax = std::max(bmax, dl.bits);
        }
      if (bmax && !sp.exact && !(stg_env && atoi(stg_env) == 0)) ss.stage_words = 64u * bmax + 4u;
      // the slices DMA'd a round ahead when the driving leaf passes >= 1/16: PG_STREAM_STAGE_PRE=1 enables it (read per
      // call, tests switch it).  Off by default: measured slower on config 3 (stream 0.602 -> 0.636 ms, r05: the
      // driving leaf's loads queue behind the slices' DMA in the wave's in-order vmcnt, so every group test waits
      // for both)
      const char* pre_env = getenv("PG_STREAM_STAGE_PRE");
      if (ss.stage_words && sp.drive_pass >= 1.0 / 16 && pre_env && atoi(pre_env) == 1 &&
          4ull * (ss.set_lds_ints + 4ull * ss.stage_words * ss.num_extra) + 16 <= 48 * 1024)
        ss.stage_pre = 1;  // (within 48 KiB of LDS per block: the 256-thread blocks stay several per CU)
    }
    ss.segs = q.segs;
    ss.items = q.items;
    ss.docs = (uint32_t*)l_docs.p;
    ss.counts = (uint32_t*)l_counts.p;
    ss.err = q.err;
    ss.stamp = q.seg_matched + (S ? S : 1) + 2;
    for (size_t k = 0; k < sp.launches.size(); k++) {
      const StreamLaunch& sl = sp.launches[k];
      ss.block_first = (const uint32_t*)(dA + sl.first_off);
      HIP_CHECK(launch_stream(ss, sl.bits, sl.blocks, s));
      if (sp.split && k + 1 == sp.split_launch) HIP_CHECK(hipEventRecord(t_ctx.ev_a, s));  // the first half's survivors
    }
    q.list_docs = ss.docs;
    q.list_counts = ss.counts;
  }
  if (is_cancelled(plan->query_id)) { (void)hipStreamSynchronize(s); return fail(PG_E_CANCELLED, "query %llu cancelled", (unsigned long long)plan->query_id); }
  if (plan->deadline_ms && now_ms() > plan->deadline_ms) { (void)hipStreamSynchronize(s); return fail(PG_E_TIMEOUT, "deadline passed"); }
  CancelSlot cancel(plan->query_id, plan->query_id != 0 || plan->deadline_ms != 0);
  q.cancel = cancel.device_ptr();
  std::vector<uint64_t> direct_matched;
  bool scan_ran = false;  // the fused scan (pg_scan.hip) was launched: the trace's FUSED_SCAN path
  if (q.num_items && part.on) {
    // radix-partitioned group-by (pg_part.hip).  Filter matching every doc and one group key: level-1 partitions
    // straight from the columns into fixed-capacity regions (part_direct), level 2 likewise (part_split2s): no
    // histogram or count pass; a region overflow (keys far from uniform over the digits) reruns the query with exact
    // offsets.  Otherwise (a filter, several keys, or that rerun) the fused scan appends 64-bit entries + the level-1
    // histogram, then part_split1 / count2 / split2 with exact offsets.  Both: per-bucket aggregation.
    bool match_all = true;
    for (uint32_t si = 0; si < S && match_all; si++) match_all = filter_is_match_all(plan, plan->segments[si].leaves);
    const char* spec_env = getenv("PG_PART_SPEC");
    // the key / value id modes of part_direct, uniform over the segments (else -2: not direct)
    int kmode = -2, vmode = part.dc == (uint32_t)kNoSlot ? -1 : -2;
    if (K == 1 && S) {
      kmode = part_id_mode(q.key_kind[0], keycols[0]);
      for (uint32_t si = 1; si < S; si++)
        if (part_id_mode(q.key_kind[0], keycols[si]) != kmode) kmode = -2;
      if (part.dc != (uint32_t)kNoSlot) {
        const uint32_t vk = q.aggs[part.dc].key_kind;
        vmode = part_id_mode(vk, aggcols[(uint64_t)part.dc * 2]);
        for (uint32_t si = 1; si < S; si++)
          if (part_id_mode(vk, aggcols[((uint64_t)si * A + part.dc) * 2]) != vmode) vmode = -2;
      }
    }
    const bool modes_ok = (kmode == 0 || kmode == 1) && (vmode >= -1 && vmode <= 1);
    // (at least 16 level-1 partitions: fixed-capacity regions of 32-bit fill counters stay far below 2^32 entries)
    const bool spec = match_all && allow_spec && K == 1 && modes_ok && part.nparts1 >= 16 &&
                      !(spec_env && atoi(spec_env) == 0);
    // PG_PART_DIRECT=1: the histogram + scatter form of level 1 from the columns (exact offsets; measured slower)
    const bool direct = !spec && match_all && getenv("PG_PART_DIRECT") && atoi(getenv("PG_PART_DIRECT")) == 1;
    const uint64_t n1 = (uint64_t)part.nparts1 * blocks, n2 = (uint64_t)part.nparts1 * part.nparts2 * kPartNB;
    const uint64_t nb = (uint64_t)part.nparts1 * part.nparts2;
    // speculative capacities: 1.25x the uniform share of the docs + slack
    const uint64_t cap1 = (part_entries + part_entries / 4) / part.nparts1 + 65536;
    const uint64_t cap2 = (cap1 + part.nparts2 - 1) / part.nparts2 + 2048;
    const size_t tb = select_temp_bytes(std::max(n1, n2) + 1);
    if (spec) {
      if ((rc = p_fill.alloc_pooled(4ull * (part.nparts1 + nb) + 16)) ||
          (rc = p_ent1.alloc_pooled(4ull * cap1 * part.nparts1 + 16)) || (rc = p_ent2.alloc_pooled(4ull * cap2 * nb + 16)))
        return rc;
      HIP_CHECK(hipMemsetAsync(p_fill.p, 0, 4ull * (part.nparts1 + nb), s));
    } else if ((!direct && ((rc = p_ent0.alloc_pooled(8 * part_entries + 16)) || (rc = p_cnt0.alloc_pooled(4ull * blocks + 16)))) ||
        (rc = p_hist1.alloc_pooled(8 * (n1 + 1))) || (rc = p_off1.alloc_pooled(8 * (n1 + 1))) ||
        (rc = p_ent1.alloc_pooled(4 * part_entries + 16)) || (rc = p_hist2.alloc_pooled(8 * (n2 + 1))) ||
        (rc = p_off2.alloc_pooled(8 * (n2 + 1))) || (rc = p_ent2.alloc_pooled(4 * part_entries + 16)) ||
        (rc = p_temp.alloc_pooled(tb))) {
      return rc;
    }
    P.dc_pop_agg = -1;
    if (t_prefetch_state && part.dc != (uint32_t)kNoSlot) {  // finalised right after (pg_execute): keep the counts
      if ((rc = P.dc_pop.alloc_pooled(4ull * G + 16))) return rc;
      P.dc_pop_agg = (int)part.dc;
    }
    unsigned long long* h1 = (unsigned long long*)p_hist1.p;
    unsigned long long* o1 = (unsigned long long*)p_off1.p;
    unsigned long long* h2 = (unsigned long long*)p_hist2.p;
    unsigned long long* o2 = (unsigned long long*)p_off2.p;
    if (!spec) {
      HIP_CHECK(hipMemsetAsync(h1 + n1, 0, 8, s));
      HIP_CHECK(hipMemsetAsync(h2 + n2, 0, 8, s));
    }
    q.group_mode = GM_PART;
    q.part_shift = part.shift1;
    q.part_vbits = part.vbits;
    q.part_nparts = part.nparts1;
    q.part_dc = part.dc;
    q.part_hist = h1;
    q.part_count = (unsigned int*)p_cnt0.p;
    q.part_base = (const unsigned long long*)(dA + off_part_base);
    q.part_out = (unsigned long long*)p_ent0.p;
    t_timing.host_compile_ms = (float)(wall_ms() - t_enter);
    if (spec || direct) {
      direct_matched.resize(S);  // every doc matches: the per-segment counts are the segments' sizes
      for (uint32_t si = 0; si < S; si++) direct_matched[si] = plan->segments[si].num_docs;
      if (S) HIP_CHECK(hipMemcpyAsync(P.seg_matched.p, direct_matched.data(), 8ull * S, hipMemcpyHostToDevice, s));
    }
    if (spec) {
      PartDirectSpec pd;
      memset(&pd, 0, sizeof(pd));
      pd.blocks = blocks;
      pd.num_items = q.num_items;
      pd.nparts1 = part.nparts1;
      pd.shift1 = part.shift1;
      pd.vbits = part.vbits;
      pd.has_val = part.dc != (uint32_t)kNoSlot;
      pd.key_kind = q.key_kind[0];
      pd.key_card = q.key_card[0];
      pd.key_base = q.key_base[0];
      pd.val_agg = part.dc;
      uint32_t kbits = 1, vbits = 1;
      for (uint32_t si = 0; si < S; si++) kbits = std::max(kbits, keycols[si].bits);
      if (pd.has_val) {
        const AggSpec& va = q.aggs[part.dc];
        pd.val_kind = va.key_kind;
        pd.val_card = va.key_card;
        pd.val_base = va.key_base;
        for (uint32_t si = 0; si < S; si++) vbits = std::max(vbits, aggcols[((uint64_t)si * A + part.dc) * 2].bits);
      }
      pd.cap1 = cap1;
      pd.segs = q.segs;
      pd.items = q.items;
      pd.fill1 = (unsigned int*)p_fill.p;
      pd.out1 = (uint32_t*)p_ent1.p;
      pd.err = q.err;
      HIP_CHECK(launch_part_direct(pd, kbits, vbits, kmode, vmode, s));
    } else if (direct) {
      PartScanSpec pss;
      memset(&pss, 0, sizeof(pss));
      pss.num_keys = K;
      pss.blocks = blocks;
      pss.num_items = q.num_items;
      pss.nparts1 = part.nparts1;
      pss.shift1 = part.shift1;
      pss.vbits = part.vbits;
      pss.val_agg = part.dc;
      pss.segs = q.segs;
      pss.items = q.items;
      for (uint32_t k = 0; k < K; k++) {
        pss.key_kind[k] = q.key_kind[k];
        pss.key_card[k] = q.key_card[k];
        pss.key_base[k] = q.key_base[k];
        pss.key_stride[k] = q.key_stride[k];
      }
      if (part.dc != (uint32_t)kNoSlot) pss.val = q.aggs[part.dc];
      pss.hist1 = h1;
      pss.off1 = o1;
      pss.out1 = (uint32_t*)p_ent1.p;
      pss.err = q.err;
      HIP_CHECK(launch_part_hist(pss, s));
      HIP_CHECK(launch_exclusive_sum((const uint64_t*)h1, (uint64_t*)o1, n1 + 1, p_temp.p, tb, s));
      HIP_CHECK(launch_part_scatter(pss, s));
    } else {
      HIP_CHECK(launch_scan(q, blocks, s));
      scan_ran = true;
      HIP_CHECK(launch_exclusive_sum((const uint64_t*)h1, (uint64_t*)o1, n1 + 1, p_temp.p, tb, s));
    }
    PartSpec ps;
    memset(&ps, 0, sizeof(ps));
    ps.nparts1 = part.nparts1;
    ps.nparts2 = part.nparts2;
    ps.vbits = part.vbits;
    ps.shift1 = part.shift1;
    ps.shift2 = part.shift2;
    ps.dc_words = part.dc_words;
    // the bitmap rows are state only a merge or value sets read: a call finalised right after (the set sizes kept in
    // dc_pop) that returns no value sets and has no other bitmap aggregation skips their 1.28 GB (config 4) of writes
    const bool rows_needed = !(P.dc_pop_agg >= 0 && !(plan->flags & PG_PLAN_VALUE_SETS) && P.bit_words == part.dc_words);
    ps.row_words = rows_needed ? P.bit_words : 0u;
    ps.dc_word = part.dc_word;
    ps.n_i64 = P.n_i64;
    ps.blocks1 = blocks;
    ps.num_groups = G;
    ps.in0 = (const unsigned long long*)p_ent0.p;
    ps.base0 = (const unsigned long long*)(dA + off_part_base);
    ps.count0 = (const unsigned int*)p_cnt0.p;
    ps.off1 = o1;
    ps.in1 = (uint32_t*)p_ent1.p;
    ps.hist2 = h2;
    ps.off2 = o2;
    ps.out2 = (uint32_t*)p_ent2.p;
    ps.i64 = (unsigned long long*)P.i64.p;
    ps.bits = (uint32_t*)P.bits.p;
    ps.dc_pop = P.dc_pop_agg >= 0 ? (uint32_t*)P.dc_pop.p : nullptr;
    // slot 0 holds the doc count only when a COUNT reads it (or there is no value set to mark presence with)
    ps.count_docs = part.dc == (uint32_t)kNoSlot ? 1u : 0u;
    for (uint32_t a = 0; a < A; a++)
      if (P.aggs[a].fn == PG_AGG_COUNT) ps.count_docs = 1u;
    ps.err = q.err;
    if (spec) {
      ps.fill1 = (const unsigned int*)p_fill.p;
      ps.fill2 = (unsigned int*)p_fill.p + part.nparts1;
      ps.cap1 = cap1;
      ps.cap2 = cap2;
      HIP_CHECK(launch_part_split2s(ps, s));
      HIP_CHECK(launch_part_aggregate(ps, s));
    } else {
      if (!direct) HIP_CHECK(launch_part_split1(ps, s));
      HIP_CHECK(launch_part_count2(ps, s));
      HIP_CHECK(launch_exclusive_sum((const uint64_t*)h2, (uint64_t*)o2, n2 + 1, p_temp.p, tb, s));
      HIP_CHECK(launch_part_split2(ps, s));
      HIP_CHECK(launch_part_aggregate(ps, s));
    }
  } else if (ix.on) {
    t_timing.host_compile_ms = (float)(wall_ms() - t_enter);
    HIP_CHECK(launch_index_count(ix.spec, ix.blocks, s));
  } else if (q.num_items && sp.on && sp.split && sp.split < q.num_items) {
    // overlapped list scan: the first half's items on the second stream as soon as their stream launch is done (its
    // blocks share the CUs with the second stream launch: 128-VGPR variant), the second half's after the stream
    t_timing.host_compile_ms = (float)(wall_ms() - t_enter);
    QuerySpec qa = q, qb = q;
    qa.num_items = sp.split;
    qb.items = q.items + sp.split;
    qb.num_items = q.num_items - sp.split;
    qb.list_docs = q.list_docs + (uint64_t)sp.split * q.list_cap;
    qb.list_counts = q.list_counts + sp.split;
    const uint32_t ga = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(qa.num_items, (uint64_t)blocks * sp.split / q.num_items));
    const uint32_t gb = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(qb.num_items, blocks > ga ? blocks - ga : 1));
    sync_on_exit.s2 = true;
    HIP_CHECK(hipStreamWaitEvent(t_ctx.s2, t_ctx.ev_a, 0));
    HIP_CHECK(launch_scan(qa, ga, t_ctx.s2, true));
    HIP_CHECK(hipEventRecord(t_ctx.ev_l, t_ctx.s2));
    HIP_CHECK(launch_scan(qb, gb, s, true));
    HIP_CHECK(hipStreamWaitEvent(s, t_ctx.ev_l, 0));  // everything after (readbacks, finalize) sees both halves
    scan_ran = true;
  } else if (q.num_items) {
    t_timing.host_compile_ms = (float)(wall_ms() - t_enter);
    HIP_CHECK(launch_scan(q, blocks, s));
    scan_ran = true;
  }
  HIP_CHECK(timing_record(ev[2], s));
  const uint64_t n_sm = (S ? S : 1) + 4;
  uint64_t* sm = (uint64_t*)t_ctx.readback.get(8ull * n_sm);
  if (!sm) return fail(PG_E_NOMEM, "pinned readback of %llu bytes failed", (unsigned long long)(8ull * n_sm));
  // the match counts + error word, and a small final state, written into mapped host memory by one launch
  CopySpans rb;
  memset(&rb, 0, sizeof(rb));
  rb.add(P.seg_matched.p, t_ctx.readback.dev(sm), 8ull * n_sm);
  P.host_state = false;
  if (t_prefetch_state && (P.mode == GM_DENSE || P.mode == GM_NONE) && !P.bit_words &&
      P.num_slots * 8ull * (P.n_i64 + 2ull * P.n_fx + P.n_min + P.n_max) <= kHostFinalBytes) {
    const uint64_t G = P.num_slots;
    const uint64_t b64 = G * 8ull * P.n_i64, bf = G * 16ull * P.n_fx, bmn = G * 8ull * P.n_min, bmx = G * 8ull * P.n_max;
    uint8_t* h = (uint8_t*)t_ctx.state_host.get(b64 + bf + bmn + bmx + 8);
    if (h) {
      const PinnedBuf& sh = t_ctx.state_host;
      if (b64) rb.add(P.i64.p, sh.dev(h), b64);
      if (bf) rb.add(P.fx.p, sh.dev(h + b64), bf);
      if (bmn) rb.add(P.mn.p, sh.dev(h + b64 + bf), bmn);
      if (bmx) rb.add(P.mx.p, sh.dev(h + b64 + bf + bmn), bmx);
      P.host_state = true;
    }
  }
  HIP_CHECK(launch_copy_spans(rb, s));
  if (plan->deadline_ms && q.cancel) {  // wait, turning a passed deadline into the kernel's stop flag
    for (;;) {
      const hipError_t e = hipStreamQuery(s);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) HIP_CHECK(e);
      if (now_ms() > plan->deadline_ms) cancel.set(2);
      sched_yield();
    }
  }
  PG_PROF("launched");
  HIP_CHECK(hipStreamSynchronize(s));
  if (cancel.state() == 1) return fail(PG_E_CANCELLED, "query %llu cancelled", (unsigned long long)plan->query_id);
  if (cancel.state() == 2) return fail(PG_E_TIMEOUT, "deadline passed during the scan");
  float pre_ms = 0, filt_ms = 0, scan_ms = 0;
  // pre-pass: ev[0] -> ev_pre; pre-filter kernels: -> ev[1]; the stream: its wall-clock stamps; the scan: the rest of
  // ev[0] -> ev[2] (with the launch boundaries between them)
  float total_ms = 0;
  if (ev_pre != ev[0]) (void)hipEventElapsedTime(&pre_ms, ev[0], ev_pre);
  if (!pre_launches.empty()) (void)hipEventElapsedTime(&filt_ms, ev_pre, ev[1]);
  (void)hipEventElapsedTime(&total_ms, ev[0], ev[2]);
  {
    const uint64_t* st = sm + (S ? S : 1) + 2;
    if (sp.on && q.num_items && st[1] && ~st[0] <= st[1] && g_wall_khz)
      filt_ms += (float)((double)(st[1] - ~st[0]) / (double)g_wall_khz);
  }
  scan_ms = std::max(0.0f, total_ms - pre_ms - filt_ms);
  (void)hipGetLastError();  // an elapsed time that could not be read (events skipped) must not stick to a later launch
  t_timing.prepass_ms = pre_ms;
  t_timing.prefilter_ms = filt_ms;
  t_timing.scan_ms = scan_ms;
  t_timing.scan_launches = (blocks || (ix.on && ix.blocks) ? 1 : 0) + (sp.on && q.num_items ? 1 : 0);  // + the stream
  t_trace.path |= (scan_ran ? PG_PATH_FUSED_SCAN : 0u) | (ix.on ? PG_PATH_INDEX_COUNT : 0u) |
                  (sp.on && q.num_items ? PG_PATH_STREAM : 0u) |
                  (part.on ? PG_PATH_PARTITIONED : 0u) | (ns_docs || ns_matched ? PG_PATH_NONSCAN : 0u) |
                  ((!pre.empty() && !ix.on) || !luts.empty() ? PG_PATH_PREPASS : 0u);
  t_trace.stream_leaf = sp.on && q.num_items ? sp.leaf : 0xFFFFFFFFu;
  t_trace.group_mode = (uint32_t)P.mode;
  t_trace.num_slots = P.num_slots;
  t_trace.num_segments_nonscan = 0;
  for (uint32_t si = 0; si < S; si++) t_trace.num_segments_nonscan += nonscan[si];
  t_trace.device_ms = pre_ms + filt_ms + scan_ms;
  memset(&stats, 0, sizeof(stats));
  stats.num_total_docs = total_docs;
  stats.num_segments_processed = S;
  stats.num_entries_scanned_in_filter = entries_in_filter;
  {
    for (uint32_t i = 0; i < S; i++) { stats.num_docs_scanned += sm[i]; stats.num_segments_matched += sm[i] > 0; }
    stats.num_docs_scanned += ns_docs;  // NonScanBasedAggregationOperator: numDocsScanned = numTotalDocs
    stats.num_segments_matched += ns_matched;
    const uint32_t err = (uint32_t)sm[S ? S : 1];
    if (err & 8u) return kRetryNoStream;     // more stream survivors than the regions hold: rerun without it
    if (err & 16u) return kRetryExactPart;   // a speculative partition region overflowed: rerun with exact offsets
    if (err & 4u) return kRetryLargerTable;  // hash table over its fill budget: rerun with a larger one
    if (err & 128u)  // pg_scan.hip mv_key_update: a doc's key tuples beyond the 16-bit first-seen position
      return fail(PG_E_UNSUPPORTED, "a doc with more than 65535 multi-value key tuples under numGroupsLimit");
    if (err & 64u)  // pg_filter.hip: the exact-mode stream kernel found its LDS LUT at a nonzero base address
      return fail(PG_E_INVALID, "stream kernel LDS layout check failed (code %u): the exact LUT is not at LDS offset 0", err);
    if (err) return fail(PG_E_INVALID, "device bounds check failed (code %u): a %s fell outside the plan's key space", err,
                         (err & 2u) && !(err & 1u) ? "DISTINCTCOUNT value" : "group key");
  }
  stats.num_entries_scanned_post_filter = (stats.num_docs_scanned - ns_docs) * P.projected_cols;
  if (P.mode == GM_HASH_SEG) {
    const double t0 = wall_ms();
    if ((rc = truncate_and_merge(P, limit, q.mv_keys != 0, s))) return rc;
    t_timing.finalize_wall_ms = (float)(wall_ms() - t0);
  }
  return PG_OK;
}


// compile_and_run with its internal retries: a larger hash table after a fill overflow, no selective stream after a
// survivor-region overflow.
int run_with_retries(const pg_plan* plan, Partials& P, pg_stats& st) {
  uint64_t cap = 0;
  bool allow_stream = true, allow_spec = true;
  for (;;) {
    const int rc = compile_and_run(plan, P, st, cap, allow_stream, allow_spec);
    if (rc == kRetryNoStream || rc == kRetryExactPart || rc == kRetryLargerTable) t_trace.reruns++;
    if (rc == kRetryNoStream) { allow_stream = false; t_trace.rerun_reasons |= PG_RERUN_STREAM; continue; }
    if (rc == kRetryExactPart) { allow_spec = false; t_trace.rerun_reasons |= PG_RERUN_PARTITION; continue; }
    if (rc != kRetryLargerTable) return rc;
    t_trace.rerun_reasons |= PG_RERUN_HASH;
    cap = P.num_slots * 8;  // the group-by hash table overflowed: rerun with 8x the slots
    if (cap > kMaxHashSlots) return fail(PG_E_UNSUPPORTED, "group-by needs more than %llu hash slots", (unsigned long long)kMaxHashSlots);
  }
}

// A plan whose packed group key cannot be formed: more keys than the scan takes, or a key-space product >= 2^62
// (DictionaryBasedGroupKeyGenerator's longOverflow, :117-131, over table-global key spaces).
bool plan_needs_wide(const pg_plan* plan) {
  if (!plan || plan->abi_version != PG_ABI_VERSION || !plan->num_keys || !plan->keys) return false;
  if (plan->num_keys > (uint32_t)kMaxKeys) return true;
  uint64_t G = 1;
  for (uint32_t k = 0; k < plan->num_keys; k++) {
    const uint64_t c = plan->keys[k].cardinality;
    if (!c) return false;  // compile_and_run reports it
    if (G > ((1ull << 62) - 1) / c) return true;
    G *= c;
  }
  return false;
}

// ArrayMapBasedHolder (DictionaryBasedGroupKeyGenerator.java:777-860) on the device: intern every doc's key tuple
// (pg_wide.hip), then run the plan grouped by the tuple slot.
int run_wide(const pg_plan* plan, Partials& P, pg_stats& st) {
  const uint32_t K = plan->num_keys, S = plan->num_segments;
  t_trace.path |= PG_PATH_WIDE_KEYS;
  if (K > kMaxWideKeys) return fail(PG_E_UNSUPPORTED, "more than %u group-by keys", kMaxWideKeys);
  if (S && !plan->segments) return fail(PG_E_INVALID, "null segment list");
  for (uint32_t k = 0; k < K; k++)
    if (!plan->keys[k].cardinality || plan->keys[k].kind > PG_KEY_KEYMAP) return fail(PG_E_INVALID, "group key %u: bad key space", k);
  int rc = t_ctx.init();
  if (rc) return rc;
  hipStream_t s = plan->stream ? (hipStream_t)plan->stream : thread_stream();
  auto W = std::make_shared<WideKeys>();
  W->K = K;
  std::vector<ColumnRes> wcols(S);
  uint64_t cap = 0;
  {
    std::shared_lock<std::shared_mutex> lk(g_seg_mu);
    std::vector<ColDesc> kc((uint64_t)S * K);
    std::vector<uint32_t> nd(S);
    uint64_t expect = 0, max_docs = 0;
    for (uint32_t si = 0; si < S; si++) {
      auto it = g_segs.find(plan->segments[si].seg_key);
      if (it == g_segs.end()) return fail(PG_E_NOTFOUND, "segment %llu not resident", (unsigned long long)plan->segments[si].seg_key);
      nd[si] = plan->segments[si].num_docs;
      max_docs = std::max<uint64_t>(max_docs, nd[si]);
      uint64_t prod = 1;
      for (uint32_t k = 0; k < K; k++) {
        const pg_key& key = plan->keys[k];
        auto ct = it->second->cols.find(key.col_id);
        const ColumnRes* c = ct == it->second->cols.end() ? nullptr : &ct->second;
        if ((rc = check_key_column(c, key, k, si))) return rc;
        if (c->num_docs < nd[si]) return fail(PG_E_INVALID, "key column %u has fewer docs than the segment", key.col_id);
        key_coldesc(kc[(uint64_t)si * K + k], c, key);
        const uint32_t kcard = c->fwd == FWD_RAW ? std::max(1u, nd[si]) : std::max(1u, c->card);
        prod = prod > nd[si] / kcard ? (uint64_t)nd[si] + 1 : prod * kcard;
      }
      expect += std::min<uint64_t>(prod, nd[si]);
      ColumnRes& w = wcols[si];
      if ((rc = w.words.alloc_pooled(((uint64_t)nd[si] + 4) * 4))) return rc;
      HIP_CHECK(hipMemsetAsync(w.words.p, 0, ((uint64_t)nd[si] + 4) * 4, s));
    }
    cap = pow2_at_least(std::max<uint64_t>(1024, 2 * expect));
    cap = std::min<uint64_t>(cap, 1ull << 26);  // grows on overflow
    std::vector<uint32_t*> outs(S);
    for (uint32_t si = 0; si < S; si++) outs[si] = (uint32_t*)wcols[si].words.p;
    std::vector<uint32_t> kkind(K), kcard(K);
    std::vector<int64_t> kbase(K);
    for (uint32_t k = 0; k < K; k++) {
      kkind[k] = plan->keys[k].kind;
      kcard[k] = plan->keys[k].cardinality;
      kbase[k] = plan->keys[k].base;
    }
    // parameter block: [ColDesc S*K][num_docs S][out S][kind K][base K][card K]
    std::vector<uint8_t> blob;
    auto put = [&](const void* p, uint64_t n) {
      const uint64_t at = (blob.size() + 15) & ~15ull;
      blob.resize(at + n);
      if (n) memcpy(&blob[at], p, n);
      return at;
    };
    const uint64_t o_kc = put(kc.data(), kc.size() * sizeof(ColDesc)), o_nd = put(nd.data(), 4ull * S),
                   o_out = put(outs.data(), 8ull * S), o_kind = put(kkind.data(), 4ull * K),
                   o_base = put(kbase.data(), 8ull * K), o_card = put(kcard.data(), 4ull * K);
    DevBuf params, tags, misc;
    if ((rc = params.alloc_pooled(blob.size()))) return rc;
    HIP_CHECK(hipMemcpyAsync(params.p, blob.data(), blob.size(), hipMemcpyHostToDevice, s));
    const uint8_t* dp = (const uint8_t*)params.p;
    if ((rc = misc.alloc_pooled(16))) return rc;
    for (;;) {
      if (cap > kMaxHashSlots || cap * (8ull + 4ull * K) > kStateBudget)
        return fail(PG_E_UNSUPPORTED, "group key tuple table of %llu slots exceeds the state budget", (unsigned long long)cap);
      if ((rc = tags.alloc_pooled(cap * 8))) return rc;
      if ((rc = W->tuples.alloc_pooled(cap * 4ull * K))) return rc;
      HIP_CHECK(hipMemsetAsync(tags.p, 0, cap * 8, s));
      HIP_CHECK(hipMemsetAsync(misc.p, 0, 16, s));
      WideSpec ws;
      memset(&ws, 0, sizeof(ws));
      ws.K = K;
      ws.num_segments = S;
      ws.max_fill = (uint32_t)(cap / 4 * 3);
      ws.mask = cap - 1;
      ws.tags = (unsigned long long*)tags.p;
      ws.tuples = (uint32_t*)W->tuples.p;
      ws.fill = (unsigned int*)misc.p;
      ws.err = (unsigned int*)misc.p + 1;
      ws.keycols = (const ColDesc*)(dp + o_kc);
      ws.num_docs = (const uint32_t*)(dp + o_nd);
      ws.out = (uint32_t* const*)(dp + o_out);
      ws.key_kind = (const uint32_t*)(dp + o_kind);
      ws.key_base = (const int64_t*)(dp + o_base);
      ws.key_card = (const uint32_t*)(dp + o_card);
      HIP_CHECK(launch_intern_tuples(ws, (uint32_t)max_docs, s));
      uint32_t fe[2] = {0, 0};
      HIP_CHECK(hipMemcpyAsync(fe, misc.p, 8, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipStreamSynchronize(s));
      if (fe[1] & 1u) return fail(PG_E_INVALID, "device bounds check failed: a key fell outside the plan's key space");
      if (!(fe[1] & 4u)) break;
      cap *= 4;  // over the fill budget: a larger table
    }
  }
  W->cap = cap;
  for (uint32_t si = 0; si < S; si++) {  // the tuple-slot column: an identity "dictionary" over [0, cap)
    ColumnRes& w = wcols[si];
    w.has_dict = true;
    w.dtype = PG_INT;
    w.card = (uint32_t)cap;
    w.imin = 0;
    w.imax = (int64_t)cap - 1;
    w.dmin = 0;
    w.dmax = (double)(cap - 1);
    w.fwd = FWD_SV;
    w.num_docs = w.num_values = plan->segments[si].num_docs;
    w.bits = 32;
    w.identity = true;
  }
  W->key1.col_id = kWideColId;
  W->key1.kind = PG_KEY_VALUE_OFFSET;
  W->key1.cardinality = (uint32_t)cap;
  W->key1.base = 0;
  pg_plan sh = *plan;
  sh.num_keys = 1;
  sh.keys = &W->key1;
  sh.num_order = 0;
  sh.order = nullptr;
  sh.limit = 0;
  t_wide_cols = &wcols;
  rc = run_with_retries(&sh, P, st);
  t_wide_cols = nullptr;
  if (hipStreamSynchronize(s) != hipSuccess && !rc) rc = fail(PG_E_HIP, "stream failed");
  if (rc) return rc;
  P.wide = W;
  // numEntriesScannedPostFilter counts the user's key columns, not the tuple column (AggregationOperator.java:84-89)
  std::unordered_set<uint32_t> proj;
  for (uint32_t a = 0; a < plan->num_aggs; a++) {
    const pg_agg& g = plan->aggs[a];
    if (g.fn == PG_AGG_COUNT) continue;
    proj.insert(g.col_a & ~PG_COL_DERIVED);
    if ((g.fn == PG_AGG_SUM || g.fn == PG_AGG_MIN || g.fn == PG_AGG_MAX || g.fn == PG_AGG_AVG) && g.op != PG_EXPR_COL)
      proj.insert(g.col_b & ~PG_COL_DERIVED);
  }
  for (uint32_t k = 0; k < K; k++) proj.insert(plan->keys[k].col_id & ~PG_COL_DERIVED);
  P.projected_cols = (uint32_t)proj.size();
  st.num_entries_scanned_post_filter = st.num_docs_scanned * P.projected_cols;
  return PG_OK;
}

struct PartialsImpl {
  Partials P;
  uint32_t ldev = 0;  // the logical device holding the state (its pg_partials_* calls run there)
};

// wide-key exchange rows carry their tuple after the state row: K uint32 table-global key ids, padded to 8 bytes
uint64_t wide_tuple_bytes(uint32_t K) { return (4ull * K + 7) & ~7ull; }

void fill_handle(pg_partials* p, PartialsImpl* impl) {
  Partials& P = impl->P;
  p->num_slots = P.num_slots;
  p->mode = P.wide ? PG_STATE_TUPLES : P.mode == GM_HASH ? PG_STATE_HASH : PG_STATE_DENSE;
  p->n_i64 = P.n_i64; p->n_fx = P.n_fx; p->n_min = P.n_min; p->n_max = P.n_max;
  p->bitmap_words = P.bit_words;
  p->layout = P.layout;
  p->fx_sig = P.fx_sig();
  p->flags = P.flags;
  p->row_bytes = row_bytes(P.view()) + (P.wide ? wide_tuple_bytes(P.wide->K) : 0);
  p->keys = (uint64_t*)P.keys.p;
  p->i64 = (int64_t*)P.i64.p;
  p->fx = (int64_t*)P.fx.p;
  p->mn = (int64_t*)P.mn.p;
  p->mx = (int64_t*)P.mx.p;
  p->bitmaps = (uint32_t*)P.bits.p;
  p->impl = impl;
}

FinalSpec make_final(const Partials& P, const pg_plan* plan) {
  FinalSpec f;
  memset(&f, 0, sizeof(f));
  f.num_aggs = (uint32_t)P.aggs.size();
  f.num_keys = (uint32_t)P.key_card.size();
  for (uint32_t a = 0; a < f.num_aggs; a++) f.aggs[a] = P.aggs[a];
  for (uint32_t k = 0; k < f.num_keys; k++) {
    f.key_card[k] = P.key_card[k];
    f.key_stride[k] = P.key_stride[k];
  }
  if (plan->num_order) {
    f.order_kind = plan->order[0].kind;
    f.order_index = plan->order[0].index;
    f.order_desc = plan->order[0].desc;
  }
  return f;
}

// The result order of nc candidates (plan's ORDER BY items, then ascending key ids, first key first) as a permutation
// in `perm`; `exact`: only its first plan->limit entries are ordered (PG_PLAN_EXACT_LIMIT keeps just those).
// key_id(i, k) = candidate i's k-th key id.
template <class KeyId>
void order_rows(const pg_plan* plan, const Partials& P, uint64_t nc, const std::vector<double>& hv,
                const std::vector<int64_t>& hc, KeyId key_id, bool exact, std::vector<uint64_t>& perm) {
  const uint32_t A = plan->num_aggs, K = plan->num_keys;
  perm.resize(nc);
  for (uint64_t i = 0; i < nc; i++) perm[i] = i;
  if (!K || !(plan->num_order || exact)) return;
  // one row of order images per candidate (ascending = ranks first): AGG items as the order-preserving image of the
  // final double, DESC items complemented, then the key ids
  const uint32_t W = plan->num_order + K;
  std::vector<uint64_t> ok(nc * W);
  for (uint64_t i = 0; i < nc; i++) {
    uint64_t* row = ok.data() + i * W;
    for (uint32_t o = 0; o < plan->num_order; o++) {
      const pg_order& it = plan->order[o];
      uint64_t x;
      if (it.kind == PG_ORDER_AGG) {
        double v = hv[i * A + it.index];
        if (P.aggs[it.index].fn == PG_AGG_AVG) {
          const int64_t c = hc[i * A + it.index];
          v = c ? v / (double)c : -INFINITY;
        }
        if (v == 0) v = 0;  // -0.0 ties with 0.0, as the double comparison does
        int64_t bits;
        memcpy(&bits, &v, 8);
        x = bits >= 0 ? ((uint64_t)bits | 0x8000000000000000ull) : ~(uint64_t)bits;
      } else {
        x = key_id(i, it.index);
      }
      row[o] = it.desc ? ~x : x;
    }
    for (uint32_t k = 0; k < K; k++) row[plan->num_order + k] = key_id(i, k);
  }
  // the order images keep only the bits in which the candidates differ (the rest is common to all of them, so the
  // order is the order of those fields): when every row's fields fit one 64-bit word, a radix sort of the packed words
  // (config 4's server trim: tens of thousands of candidates, 440 -> ~30 us) instead of a comparison sort of rows
  uint32_t lo[64], wd[64], total = W <= 64 ? 0u : 65u;
  for (uint32_t w = 0; w < W && total <= 64; w++) {
    uint64_t any = 0, all = ~0ull;
    for (uint64_t i = 0; i < nc; i++) { any |= ok[i * W + w]; all &= ok[i * W + w]; }
    const uint64_t diff = any & ~all;
    lo[w] = diff ? (uint32_t)__builtin_ctzll(diff) : 0u;
    wd[w] = diff ? 64u - (uint32_t)__builtin_clzll(diff) - lo[w] : 0u;
    total += wd[w];
  }
  if (total <= 64 && nc > 64) {
    std::vector<uint64_t> pk(nc), pk2(nc);
    std::vector<uint64_t> p2(nc);
    for (uint64_t i = 0; i < nc; i++) {
      uint64_t x = 0;
      for (uint32_t w = 0; w < W; w++)
        if (wd[w]) x = (wd[w] == 64 ? 0 : x << wd[w]) | ((ok[i * W + w] >> lo[w]) & (wd[w] == 64 ? ~0ull : (1ull << wd[w]) - 1));
      pk[i] = x;
    }
    // LSD radix sort, 11-bit digits over the packed width (stable: equal words keep candidate order)
    for (uint32_t sh = 0; sh < total; sh += 11) {
      uint32_t cnt[2049] = {0};
      for (uint64_t i = 0; i < nc; i++) cnt[((pk[i] >> sh) & 2047u) + 1]++;
      for (uint32_t d = 0; d < 2048; d++) cnt[d + 1] += cnt[d];
      for (uint64_t i = 0; i < nc; i++) {
        const uint32_t d = (uint32_t)((pk[i] >> sh) & 2047u);
        pk2[cnt[d]] = pk[i];
        p2[cnt[d]++] = perm[i];
      }
      pk.swap(pk2);
      perm.swap(p2);
    }
    return;
  }
  auto before = [&](uint64_t i, uint64_t j) {
    const uint64_t *x = ok.data() + i * W, *y = ok.data() + j * W;
    for (uint32_t w = 0; w < W; w++)
      if (x[w] != y[w]) return x[w] < y[w];
    return false;
  };
  if (exact && nc > plan->limit) std::partial_sort(perm.begin(), perm.begin() + plan->limit, perm.end(), before);
  else std::sort(perm.begin(), perm.end(), before);
}

int build_result(pg_partials* pp, const pg_plan* plan, pg_result** out, const Partials& P, uint64_t nc,
                 const std::vector<uint64_t>& hk, const std::vector<double>& hv, const std::vector<int64_t>& hc,
                 bool sets, const std::vector<uint64_t>& hoff, const uint32_t* hids, uint64_t n_ids, uint64_t merged);


// finalize() for small dense states without DISTINCTCOUNT: the same groups, final values and ORDER BY candidates
// (ties with the limit-th on the first ORDER BY item included) as the device path, computed from a host copy.
int finalize_small(pg_partials* pp, const pg_plan* plan, pg_result** out, const Partials& P, const FinalSpec& f,
                   hipEvent_t e0, hipEvent_t e1, hipStream_t s) {
  const StateView v = P.view();
  const uint32_t A = plan->num_aggs, K = plan->num_keys;
  const uint64_t G = P.num_slots;
  const uint64_t b64 = G * 8ull * v.n_i64, bf = G * 16ull * v.n_fx, bmn = G * 8ull * v.n_min, bmx = G * 8ull * v.n_max;
  uint8_t* h;
  if (P.host_state) {  // copied back with the scan's match counts (pg_execute): no device work left
    h = (uint8_t*)t_ctx.state_host.p;
    t_timing.finalize_ms = 0;
  } else {
    h = (uint8_t*)t_ctx.readback.get(b64 + bf + bmn + bmx + 8);
    if (!h) return fail(PG_E_NOMEM, "pinned readback failed");
    HIP_CHECK(hipMemcpyAsync(h, v.i64, b64, hipMemcpyDeviceToHost, s));
    if (bf) HIP_CHECK(hipMemcpyAsync(h + b64, v.fx, bf, hipMemcpyDeviceToHost, s));
    if (bmn) HIP_CHECK(hipMemcpyAsync(h + b64 + bf, v.mn, bmn, hipMemcpyDeviceToHost, s));
    if (bmx) HIP_CHECK(hipMemcpyAsync(h + b64 + bf + bmn, v.mx, bmx, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipEventRecord(e1, s));
    HIP_CHECK(hipStreamSynchronize(s));
    float fm = 0;
    (void)hipEventElapsedTime(&fm, e0, e1);
    t_timing.finalize_ms = fm;
  }
  const uint64_t* i64 = (const uint64_t*)h;
  const uint64_t* fx = (const uint64_t*)(h + b64);
  const int64_t* mn = (const int64_t*)(h + b64 + bf);
  const int64_t* mx = (const int64_t*)(h + b64 + bf + bmn);
  // 1. the groups (aggregation-only: slot 0, always one row) and 2. their final values (final_values_kernel)
  std::vector<uint64_t> hk;
  std::vector<double> hv;
  std::vector<int64_t> hc;
  for (uint64_t sl = 0; sl < G; sl++) {
    const int64_t count = (int64_t)i64[sl * v.n_i64];
    if (K && count <= 0) continue;
    hk.push_back(sl);
    for (uint32_t a = 0; a < A; a++) {
      const AggSpec& g = f.aggs[a];
      double x = 0;
      int64_t c = 0;
      switch (g.fn) {
        case PG_AGG_COUNT: x = (double)count; break;
        case PG_AGG_COUNTMV: x = (double)(int64_t)i64[sl * v.n_i64 + g.slot]; break;
        case PG_AGG_SUM:
        case PG_AGG_AVG:
          if (g.integer) {
            x = (double)(int64_t)i64[sl * v.n_i64 + g.slot];
          } else {
            const uint64_t* w = fx + (sl * v.n_fx + g.slot) * 2;
            x = fx_final(g, w, g.sp_min != kNoSp ? mn[sl * v.n_min + g.sp_min] : 0,
                         g.sp_max != kNoSp ? mx[sl * v.n_max + g.sp_max] : 0);
          }
          if (g.fn == PG_AGG_AVG) c = g.cnt_slot ? (int64_t)i64[sl * v.n_i64 + g.cnt_slot] : count;
          break;
        case PG_AGG_MIN: x = order_key_decode(mn[sl * v.n_min + g.slot]); break;
        case PG_AGG_MAX: x = order_key_decode(mx[sl * v.n_max + g.slot]); break;
      }
      hv.push_back(x);
      hc.push_back(c);
    }
    if (!K) break;
  }
  uint64_t nc = hk.size();
  const uint64_t merged = nc;
  // 3. ORDER BY trim: the candidates whose first-ORDER-BY image is <= the limit-th smallest (order_keys_kernel)
  if (K && plan->num_order && plan->limit && nc > plan->limit) {
    std::vector<uint64_t> ok(nc);
    for (uint64_t i = 0; i < nc; i++) {
      uint64_t o;
      if (f.order_kind == PG_ORDER_KEY) {
        o = (hk[i] / f.key_stride[f.order_index]) % f.key_card[f.order_index];
      } else {
        const uint32_t a = f.order_index;
        double x = hv[i * A + a];
        if (f.aggs[a].fn == PG_AGG_AVG) { const int64_t c = hc[i * A + a]; x = c ? x / (double)c : -INFINITY; }
        int64_t b;
        memcpy(&b, &x, 8);
        o = b >= 0 ? ((uint64_t)b | 0x8000000000000000ull) : ~(uint64_t)b;
      }
      ok[i] = f.order_desc ? ~o : o;
    }
    std::vector<uint64_t> srt(ok);
    std::nth_element(srt.begin(), srt.begin() + (plan->limit - 1), srt.end());
    const uint64_t t = srt[plan->limit - 1];
    uint64_t w = 0;
    for (uint64_t i = 0; i < nc; i++) {
      if (ok[i] > t) continue;
      hk[w] = hk[i];
      for (uint32_t a = 0; a < A; a++) { hv[w * A + a] = hv[i * A + a]; hc[w * A + a] = hc[i * A + a]; }
      w++;
    }
    nc = w;
    hk.resize(nc);
    hv.resize(nc * A);
    hc.resize(nc * A);
  }
  return build_result(pp, plan, out, P, nc, hk, hv, hc, false, {}, nullptr, 0, merged);
}

// Partial state -> host result: the groups present (doc count > 0), their final values, the plan's ORDER BY trim
// (IndexedTable.finish -> TableResizer.getTopRecords: a radix sort on the first ORDER BY item on the device, the
// candidates -- every group that ranks within `limit`, ties included -- fully ordered on the host) and, on request,
// the DISTINCTCOUNT value sets.
int finalize_core(pg_partials* pp, const pg_plan* plan, pg_result** out);

// Wide-key partials: the state is keyed by tuple slot, so the device part runs on the plan's one-key form (a leading
// ORDER BY on an aggregation still trims on the device; one on a key cannot, every group comes back) and build_result
// maps slots to tuples and orders by the caller's full ORDER BY.
int finalize(pg_partials* pp, const pg_plan* plan, pg_result** out) {
  Partials& P = ((PartialsImpl*)pp->impl)->P;
  if (!P.wide) return finalize_core(pp, plan, out);
  if (plan->num_keys != P.wide->K) return fail(PG_E_INVALID, "plan does not match partials");
  if (plan->num_order && !plan->order) return fail(PG_E_INVALID, "null order list");
  for (uint32_t i = 0; i < plan->num_order; i++) {
    const pg_order& o = plan->order[i];
    if (o.kind > PG_ORDER_KEY || (o.kind == PG_ORDER_AGG && o.index >= plan->num_aggs) ||
        (o.kind == PG_ORDER_KEY && o.index >= plan->num_keys))
      return fail(PG_E_INVALID, "bad ORDER BY item %u", i);
  }
  pg_plan sh = *plan;
  sh.num_keys = 1;
  sh.keys = &P.wide->key1;
  pg_order o0{};
  if (plan->num_order && plan->order[0].kind == PG_ORDER_AGG) {
    o0 = plan->order[0];
    sh.num_order = 1;
    sh.order = &o0;
  } else {
    sh.num_order = 0;
    sh.order = nullptr;
    sh.limit = 0;
  }
  P.wide->user_plan = plan;
  const int rc = finalize_core(pp, &sh, out);
  P.wide->user_plan = nullptr;
  return rc;
}

int finalize_core(pg_partials* pp, const pg_plan* plan, pg_result** out) {
  const double t0 = wall_ms();
  struct Stamp {
    double t0;
    ~Stamp() { t_timing.finalize_wall_ms = (float)(wall_ms() - t0); }
  } stamp{t0};
  PartialsImpl* impl = (PartialsImpl*)pp->impl;
  Partials& P = impl->P;
  const uint32_t A = plan->num_aggs, K = plan->num_keys;
  if (A != P.aggs.size() || K != P.key_card.size()) return fail(PG_E_INVALID, "plan does not match partials");
  if (plan->num_order && !plan->order) return fail(PG_E_INVALID, "null order list");
  for (uint32_t i = 0; i < plan->num_order; i++) {
    const pg_order& o = plan->order[i];
    if (o.kind > PG_ORDER_KEY || (o.kind == PG_ORDER_AGG && o.index >= A) || (o.kind == PG_ORDER_KEY && o.index >= K))
      return fail(PG_E_INVALID, "bad ORDER BY item %u", i);
  }
  int rc = t_ctx.init();
  if (rc) return rc;
  hipStream_t s = thread_stream();
  hipEvent_t e0 = t_ctx.ev[3], e1 = t_ctx.ev[2];
  const StateView v = P.view();
  const FinalSpec f = make_final(P, plan);
  const uint32_t AA = A ? A : 1;

  bool any_dc = false;
  for (uint32_t a = 0; a < A; a++) any_dc |= P.aggs[a].fn == PG_AGG_DISTINCTCOUNT;
  const uint64_t row_words = (uint64_t)v.n_i64 + 2ull * v.n_fx + v.n_min + v.n_max;
  if ((P.mode == GM_DENSE || P.mode == GM_NONE) && !any_dc && P.num_slots * row_words * 8 <= kHostFinalBytes) {
    if (!P.host_state) HIP_CHECK(hipEventRecord(e0, s));  // (a state already on the host needs no device time)
    return finalize_small(pp, plan, out, P, f, e0, e1, s);
  }
  HIP_CHECK(hipEventRecord(e0, s));
  Scratch sc(s);

  // 0. a trim ordered by a DISTINCTCOUNT whose set sizes the bucket pass kept (config 4's server trim): the candidates
  // straight from a histogram of the sizes and one select pass, their final values, then on to the value sets
  // (PG_TRIM_POP=0: the general path below)
  const char* tp_env = getenv("PG_TRIM_POP");
  const bool pop_trim = K && plan->num_order && plan->limit && P.num_slots >= kTrimSelectMinGroups && v.dc_pop &&
                        f.order_kind == PG_ORDER_AGG && f.order_index < A && v.dc_pop_agg == f.order_index &&
                        f.aggs[f.order_index].fn == PG_AGG_DISTINCTCOUNT && f.aggs[f.order_index].key_card < 8192 &&
                        !(tp_env && atoi(tp_env) == 0);
  uint64_t nc = 0, merged = 0;  // merged: the groups present before the trim
  const uint64_t* ck = nullptr;
  const double* cv = nullptr;
  const int64_t* cc = nullptr;
  const uint32_t* cs = nullptr;
  bool have_candidates = false;
  if (pop_trim) {
    const uint32_t maxv = f.aggs[f.order_index].key_card;  // set sizes are <= the value space
    unsigned int* hist = sc.get<unsigned int>(maxv + 2, rc);
    unsigned int* d_cnt = sc.get<unsigned int>(2, rc);
    if (rc) return rc;
    unsigned int* hh = (unsigned int*)t_ctx.readback.get(4ull * (maxv + 1));
    if (!hh) return fail(PG_E_NOMEM, "pinned readback failed");
    HIP_CHECK(hipMemsetAsync(hist, 0, 4ull * (maxv + 1), s));
    HIP_CHECK(hipMemsetAsync(d_cnt, 0, 4, s));
    HIP_CHECK(launch_pop_hist(v, maxv, hist, s));
    HIP_CHECK(hipMemcpyAsync(hh, hist, 4ull * (maxv + 1), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    uint64_t present = 0;
    for (uint32_t x = 0; x <= maxv; x++) present += hh[x];
    merged = present;
    if (present > plan->limit) {
      // the limit-th group's size in the ORDER BY direction; every group tied with it stays a candidate
      uint64_t cum = 0;
      uint32_t t = 0;
      if (f.order_desc) {
        for (uint32_t x = maxv + 1; x-- > 0;) { cum += hh[x]; if (cum >= plan->limit) { t = x; break; } }
      } else {
        for (uint32_t x = 0; x <= maxv; x++) { cum += hh[x]; if (cum >= plan->limit) { t = x; break; } }
      }
      uint32_t* gs = sc.get<uint32_t>(cum + 1, rc);
      uint64_t* gk = sc.get<uint64_t>(cum + 1, rc);
      double* gv = sc.get<double>((cum + 1) * AA, rc);
      int64_t* gc = sc.get<int64_t>((cum + 1) * AA, rc);
      if (rc) return rc;
      HIP_CHECK(launch_select_pop(v, t, maxv, f.order_desc != 0, gs, d_cnt, s));
      HIP_CHECK(launch_final_values(v, f, gs, cum, gk, gv, gc, s));
      nc = cum;
      ck = gk; cv = gv; cc = gc; cs = gs;
      have_candidates = true;
      PG_PROF("f_pop");
    }
  }
  if (!have_candidates) {
    // 1. the groups
    uint64_t n = 1;
    // aggregation-only: slot 0 (always one row); a merged hash state holds key 0 only if some rank had matches
    const bool single = K == 0 && P.mode != GM_HASH;
    uint32_t* slots = sc.get<uint32_t>(single ? 1 : P.num_slots, rc);
    uint32_t* d_num = sc.get<uint32_t>(2, rc);
    if (rc) return rc;
    if (single) {
      HIP_CHECK(hipMemsetAsync(slots, 0, 4, s));
    } else {
      // an ORDER BY trim re-orders the candidates anyway (build_result): a large state's present slots may come in any
      // order, by one pass with a wave-aggregated append instead of the ordered (two-pass) select
      const bool trims = K && plan->num_order && plan->limit && P.num_slots >= kTrimSelectMinGroups;
      if (trims) {
        HIP_CHECK(hipMemsetAsync(d_num, 0, 4, s));
        HIP_CHECK(launch_select_present_unordered(v, slots, (unsigned int*)d_num, s));
      } else {
        const size_t tb = select_temp_bytes(P.num_slots);
        void* temp = sc.get<uint8_t>(tb, rc);
        if (rc) return rc;
        HIP_CHECK(launch_select_slots(v, SEL_PRESENT, 0, 1, slots, d_num, temp, tb, s));
      }
      uint32_t n32 = 0;
      if ((rc = read_back(d_num, n32, s))) return rc;
      n = n32;
    }
    merged = n;
    PG_PROF("f_groups");
    // 2. final values (a radix-select trim orders the groups by an image read straight from the state, and computes the
    // final values of its candidates only)
    const bool trim = K && plan->num_order && plan->limit && n > plan->limit;
    const char* sel_env = getenv("PG_TRIM_SELECT");  // 0: always sort, 1: always select (tests), else by size
    const int sel = sel_env ? atoi(sel_env) : -1;
    const bool select = trim && (sel == 1 || (sel != 0 && n >= kTrimSelectMinGroups));
    const bool late_values = select && order_keys_from_state_ok(v, f);
    uint64_t* dkeys = nullptr;
    double* dvals = nullptr;
    int64_t* dcnts = nullptr;
    if (!late_values) {
      dkeys = sc.get<uint64_t>(n + 1, rc);
      dvals = sc.get<double>((n + 1) * AA, rc);
      dcnts = sc.get<int64_t>((n + 1) * AA, rc);
      if (rc) return rc;
      HIP_CHECK(launch_final_values(v, f, slots, n, dkeys, dvals, dcnts, s));
    }
    // 3. ORDER BY trim
    nc = n;
    ck = dkeys;
    cv = dvals;
    cc = dcnts;
    cs = slots;
    if (trim) {
      uint64_t* okeys = sc.get<uint64_t>(n, rc);
      uint64_t* skeys = sc.get<uint64_t>(n, rc);
      uint32_t* pos = sc.get<uint32_t>(n, rc);
      uint32_t* spos = sc.get<uint32_t>(n, rc);
      uint64_t* d_nc = sc.get<uint64_t>(1, rc);
      KeySpan* d_span = sc.get<KeySpan>(1, rc);
      if (rc) return rc;
      // the sort covers only the key bits that differ between groups (config 4: a DISTINCTCOUNT <= 1 000 varies in
      // 21 of the double image's 64 bits: 3 radix passes instead of 8)
      if (late_values) HIP_CHECK(launch_order_keys_state(v, f, slots, n, okeys, pos, (uint64_t*)d_span, s));
      else HIP_CHECK(launch_order_keys(f, dkeys, dvals, dcnts, n, okeys, pos, s, (uint64_t*)d_span));
      KeySpan span{};
      if ((rc = read_back(d_span, span, s))) return rc;
      PG_PROF("f_okeys");
      const uint64_t diff = span.any & span.anyz;
      const uint32_t b0 = diff ? (uint32_t)__builtin_ctzll(diff) : 0u, b1 = diff ? 64u - (uint32_t)__builtin_clzll(diff) : 1u;
      if (select) {
        // radix select of the limit-th smallest key (a histogram readback per <= 8-bit digit of the differing bits),
        // then the positions of every key up to it: no sort of all n groups
        const uint32_t W = b1 - b0;
        constexpr uint32_t kHB = 4u << kOkeyDigitBits;  // histogram bytes of the widest digit
        unsigned int* hist = sc.get<unsigned int>(kHB / 4, rc);
        unsigned int* hh = (unsigned int*)t_ctx.readback.get(kHB);
        if (rc) return rc;
        if (!hh) return fail(PG_E_NOMEM, "pinned readback failed");
        uint64_t need = plan->limit, prefix = 0;
        for (uint32_t hi = W; hi > 0;) {
          const uint32_t lo = hi > kOkeyDigitBits ? hi - kOkeyDigitBits : 0;
          const size_t hb = 4ull << (hi - lo);
          HIP_CHECK(hipMemsetAsync(hist, 0, hb, s));
          HIP_CHECK(launch_okey_hist(okeys, n, b0, W, lo, hi, prefix, hist, s));
          HIP_CHECK(hipMemcpyAsync(hh, hist, hb, hipMemcpyDeviceToHost, s));
          HIP_CHECK(hipStreamSynchronize(s));
          uint64_t cum = 0;
          uint32_t d = 0;
          const uint32_t nd = 1u << (hi - lo);
          for (; d + 1 < nd && cum + hh[d] < need; d++) cum += hh[d];
          need -= cum;
          prefix = (prefix << (hi - lo)) | d;
          hi = lo;
        }
        unsigned long long* d_cnt = (unsigned long long*)d_nc;
        HIP_CHECK(hipMemsetAsync(d_cnt, 0, 8, s));
        PG_PROF("f_radix");
        HIP_CHECK(launch_okey_select(okeys, n, b0, W, prefix, spos, d_cnt, s));
        if ((rc = read_back(d_nc, nc, s))) return rc;
        PG_PROF("f_cut");
      } else {
        const size_t tb = sort_temp_bytes(n, b0, b1);
        void* temp = sc.get<uint8_t>(tb, rc);
        if (rc) return rc;
        HIP_CHECK(launch_sort_pairs(okeys, skeys, pos, spos, n, temp, tb, s, b0, b1));
        HIP_CHECK(launch_cutoff(skeys, n, plan->limit, d_nc, s));
        if ((rc = read_back(d_nc, nc, s))) return rc;
      }
      uint64_t* gk = sc.get<uint64_t>(nc + 1, rc);
      double* gv = sc.get<double>((nc + 1) * AA, rc);
      int64_t* gc = sc.get<int64_t>((nc + 1) * AA, rc);
      uint32_t* gs = sc.get<uint32_t>(nc + 1, rc);
      if (rc) return rc;
      if (late_values) {  // the candidates' slots, then their final values
        HIP_CHECK(launch_gather_slots(slots, spos, nc, gs, s));
        HIP_CHECK(launch_final_values(v, f, gs, nc, gk, gv, gc, s));
      } else {
        HIP_CHECK(launch_gather_final(A, spos, nc, dkeys, dvals, dcnts, slots, gk, gv, gc, gs, s));
      }
      ck = gk; cv = gv; cc = gc; cs = gs;
    }
  }
  std::vector<uint64_t> hk(nc);
  std::vector<double> hv(nc * A);
  std::vector<int64_t> hc(nc * A);
  if (nc) {
    HIP_CHECK(hipMemcpyAsync(hk.data(), ck, nc * 8, hipMemcpyDeviceToHost, s));
    if (A) {
      HIP_CHECK(hipMemcpyAsync(hv.data(), cv, nc * A * 8, hipMemcpyDeviceToHost, s));
      HIP_CHECK(hipMemcpyAsync(hc.data(), cc, nc * A * 8, hipMemcpyDeviceToHost, s));
    }
  }
  // 4. value sets
  bool sets = false;
  for (uint32_t a = 0; a < A; a++) sets |= (plan->flags & PG_PLAN_VALUE_SETS) && P.aggs[a].fn == PG_AGG_DISTINCTCOUNT;
  if (sets && !P.wide && K && (plan->flags & PG_PLAN_EXACT_LIMIT) && plan->limit && nc > plan->limit) {
    // an exact limit keeps `limit` of the candidates: order them now and extract the value sets of those only (the
    // server trim of config 4 keeps 5 000 of the tens of thousands of groups tied at the boundary's set size)
    std::vector<uint32_t> hs(nc);
    HIP_CHECK(hipMemcpyAsync(hs.data(), cs, nc * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    PG_PROF("f_cands");
    std::vector<uint64_t> perm;
    order_rows(plan, P, nc, hv, hc, [&](uint64_t i, uint32_t k) { return (hk[i] / P.key_stride[k]) % P.key_card[k]; },
               true, perm);
    const uint64_t m = plan->limit;
    std::vector<uint64_t> kk(m);
    std::vector<double> kv(m * A);
    std::vector<int64_t> kc(m * A);
    std::vector<uint32_t> kslot(m);
    for (uint64_t o = 0; o < m; o++) {
      const uint64_t i = perm[o];
      kk[o] = hk[i];
      kslot[o] = hs[i];
      for (uint32_t a = 0; a < A; a++) { kv[o * A + a] = hv[i * A + a]; kc[o * A + a] = hc[i * A + a]; }
    }
    uint32_t* ks = sc.get<uint32_t>(m, rc);
    if (rc) return rc;
    HIP_CHECK(hipMemcpyAsync(ks, kslot.data(), m * 4, hipMemcpyHostToDevice, s));
    HIP_CHECK(hipStreamSynchronize(s));  // kslot is a local of this block
    hk.swap(kk);
    hv.swap(kv);
    hc.swap(kc);
    cs = ks;
    nc = m;
    PG_PROF("f_precut");
  }
  std::vector<uint64_t> hoff;
  const uint32_t* hids = nullptr;  // the value sets' ids, copied back into pinned memory (config 4: 2.5 MB)
  uint64_t n_ids = 0;
  if (sets) {
    const uint64_t m = nc * A;
    uint64_t* sizes = sc.get<uint64_t>(m + 1, rc);
    uint64_t* offs = sc.get<uint64_t>(m + 1, rc);
    const size_t tb = select_temp_bytes(m + 1);
    void* temp = sc.get<uint8_t>(tb, rc);
    if (rc) return rc;
    HIP_CHECK(hipMemsetAsync(sizes + m, 0, 8, s));
    HIP_CHECK(launch_set_sizes(v, f, cs, nc, sizes, s));
    HIP_CHECK(launch_exclusive_sum(sizes, offs, m + 1, temp, tb, s));
    hoff.resize(m + 1);
    HIP_CHECK(hipMemcpyAsync(hoff.data(), offs, (m + 1) * 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    uint32_t* ids = sc.get<uint32_t>(hoff[m] + 1, rc);
    if (rc) return rc;
    HIP_CHECK(launch_set_extract(v, f, cs, nc, offs, ids, s));
    n_ids = hoff[m];
    uint32_t* h = (uint32_t*)t_ctx.ids_host.get(n_ids * 4 + 4);
    if (!h) return fail(PG_E_NOMEM, "pinned readback of %llu set ids failed", (unsigned long long)n_ids);
    if (n_ids) HIP_CHECK(hipMemcpyAsync(h, ids, n_ids * 4, hipMemcpyDeviceToHost, s));
    hids = h;
  }
  HIP_CHECK(hipEventRecord(e1, s));
  HIP_CHECK(hipStreamSynchronize(s));
  PG_PROF("f_sets");
  float fm = 0;
  (void)hipEventElapsedTime(&fm, e0, e1);
  t_timing.finalize_ms = fm;
  return build_result(pp, plan, out, P, nc, hk, hv, hc, sets, hoff, hids, n_ids, merged);
}

// Host order of the candidates (every ORDER BY item, then the packed key: a total order) and the result rows.
// Result arrays (pg_result_free returns them): a 16-byte header holds the block's capacity; blocks of >= 256 KiB go
// back to a small cache instead of free() -- a fresh multi-MB malloc is an mmap whose pages fault on first touch
// (config 4's 2.5 MB of value-set ids cost ~0.2 ms per query that way).
constexpr uint64_t kResCacheMin = 256 * 1024;
std::mutex g_res_mu;
std::vector<uint8_t*> g_res_cache;
void* res_alloc(uint64_t n) {
  n = n ? n : 1;
  uint64_t cap = 0;
  uint8_t* b = nullptr;
  if (n >= kResCacheMin) {
    cap = kResCacheMin;
    while (cap < n) cap <<= 1;
    std::lock_guard<std::mutex> g(g_res_mu);
    for (size_t i = 0; i < g_res_cache.size(); i++) {
      const uint64_t c = *(const uint64_t*)g_res_cache[i];
      if (c >= n && c <= 4 * cap) { b = g_res_cache[i]; g_res_cache.erase(g_res_cache.begin() + (long)i); cap = c; break; }
    }
  }
  if (!b) b = (uint8_t*)malloc((cap ? cap : n) + 16);
  if (!b) return nullptr;
  *(uint64_t*)b = cap;
  return b + 16;
}
void res_free(void* p) {
  if (!p) return;
  uint8_t* b = (uint8_t*)p - 16;
  if (*(const uint64_t*)b) {
    std::lock_guard<std::mutex> g(g_res_mu);
    if (g_res_cache.size() < 8) { g_res_cache.push_back(b); return; }
  }
  free(b);
}

int build_result(pg_partials* pp, const pg_plan* plan, pg_result** out, const Partials& P, uint64_t nc,
                 const std::vector<uint64_t>& hk, const std::vector<double>& hv, const std::vector<int64_t>& hc,
                 bool sets, const std::vector<uint64_t>& hoff, const uint32_t* hids, uint64_t n_ids, uint64_t merged) {
  if (P.wide && P.wide->user_plan) plan = P.wide->user_plan;  // the caller's K keys and ORDER BY
  const uint32_t A = plan->num_aggs, K = plan->num_keys;
  const uint32_t AA = A ? A : 1;
  // key ids of candidate i: from the packed key, or (wide keys) from the tuple of its slot
  std::vector<uint32_t> wk;
  if (P.wide && nc) {
    hipStream_t s = thread_stream();
    Scratch sc(s);
    int rc = PG_OK;
    uint64_t* dk = sc.get<uint64_t>(nc, rc);
    uint32_t* dt = sc.get<uint32_t>(nc * K, rc);
    if (rc) return rc;
    wk.resize(nc * K);
    HIP_CHECK(hipMemcpyAsync(dk, hk.data(), nc * 8, hipMemcpyHostToDevice, s));
    HIP_CHECK(launch_gather_tuples((const uint32_t*)P.wide->tuples.p, K, dk, nc, dt, s));
    HIP_CHECK(hipMemcpyAsync(wk.data(), dt, nc * K * 4ull, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
  auto key_id = [&](uint64_t i, uint32_t k) -> uint64_t {
    return P.wide ? (uint64_t)wk[i * K + k] : (hk[i] / P.key_stride[k]) % P.key_card[k];
  };
  const bool exact = K && (plan->flags & PG_PLAN_EXACT_LIMIT) && plan->limit && nc > plan->limit;
  std::vector<uint64_t> perm;
  order_rows(plan, P, nc, hv, hc, key_id, exact, perm);
  // PG_PLAN_EXACT_LIMIT: the first `limit` rows of that order (the server result / the per-segment trim)
  if (exact) nc = plan->limit;

  pg_result* r = (pg_result*)calloc(1, sizeof(pg_result));
  if (!r) return fail(PG_E_NOMEM, "out of host memory");
  r->stats = pp->stats;  // local, or merged across ranks by the caller before finalize
  r->num_groups_merged = K ? merged : nc;
  r->flags = pp->flags & (PG_RESULT_GROUPS_LIMIT_REACHED | PG_RESULT_TRIM_THRESHOLD_REACHED);
  // the reference's ConcurrentIndexedTable resizes whenever it holds >= trimThreshold records: before its first resize
  // it holds every merged key, so a resize happened iff the merged groups reach the threshold
  if (K && plan->num_order && plan->trim_threshold && merged >= plan->trim_threshold)
    r->flags |= PG_RESULT_TRIM_THRESHOLD_REACHED;
  r->num_keys = K;
  r->num_aggs = A;
  r->num_groups = nc;
  r->keys = (uint32_t*)res_alloc((nc * (K ? K : 1) + 1) * 4);
  r->values = (double*)res_alloc((nc * AA + 1) * 8);
  r->counts = (int64_t*)res_alloc((nc * AA + 1) * 8);
  if (!r->keys || !r->values || !r->counts) { pg_result_free(r); return fail(PG_E_NOMEM, "out of host memory"); }
  for (uint64_t o = 0; o < nc; o++) {
    const uint64_t i = perm[o];
    for (uint32_t k = 0; k < K; k++) r->keys[o * K + k] = (uint32_t)key_id(i, k);
    for (uint32_t a = 0; a < A; a++) {
      r->values[o * A + a] = hv[i * A + a];
      r->counts[o * A + a] = hc[i * A + a];
    }
  }
  if (sets) {
    const uint64_t m = nc * A;
    r->num_distinct = n_ids;
    r->distinct_offsets = (uint64_t*)res_alloc((m + 1) * 8);
    r->distinct_ids = (uint32_t*)res_alloc(n_ids * 4 + 4);
    if (!r->distinct_offsets || !r->distinct_ids) { pg_result_free(r); return fail(PG_E_NOMEM, "out of host memory"); }
    uint64_t at = 0;
    for (uint64_t o = 0; o < nc; o++)
      for (uint32_t a = 0; a < A; a++) {
        const uint64_t src = perm[o] * A + a;
        r->distinct_offsets[o * A + a] = at;
        const uint64_t len = hoff[src + 1] - hoff[src];
        if (len) memcpy(r->distinct_ids + at, hids + hoff[src], len * 4);
        at += len;
      }
    r->distinct_offsets[m] = at;
    r->num_distinct = at;  // the kept groups' ids (an exact limit may drop candidates)
  }
  *out = r;
  return PG_OK;
}

// ---------------------------------------------------------------------------------------- relocatable plan image

static_assert(sizeof(pg_image_header) == 120 && sizeof(pg_image_segment) == 24 && sizeof(pg_image_leaf) == 88,
              "pg_image_* layouts are part of the ABI");
static_assert(sizeof(pg_image_leaf) == sizeof(pg_leaf) && offsetof(pg_image_leaf, ids_off) == offsetof(pg_leaf, ids) &&
                  offsetof(pg_image_leaf, values_off) == offsetof(pg_leaf, values) &&
                  offsetof(pg_image_leaf, num_values) == offsetof(pg_leaf, num_values),
              "a pg_image_leaf is a pg_leaf with offsets for pointers");

// A pg_plan whose pointers point into a validated image (pg_execute_image): the image is borrowed for the call.
struct PlanImage {
  pg_plan plan{};
  std::vector<pg_segment_ref> segs;
  std::vector<pg_leaf> leaves;
};

int decode_image(const void* image, uint64_t n, PlanImage& out) {
  if (!image) return fail(PG_E_INVALID, "image: null buffer");
  if ((uintptr_t)image & 7) return fail(PG_E_INVALID, "image: buffer not 8-byte aligned");
  if (n < sizeof(pg_image_header)) return fail(PG_E_INVALID, "image: %llu bytes < header", (unsigned long long)n);
  const uint8_t* base = (const uint8_t*)image;
  const pg_image_header& h = *(const pg_image_header*)image;
  if (h.magic != PG_IMAGE_MAGIC) return fail(PG_E_INVALID, "image: bad magic 0x%08x", h.magic);
  if (h.abi_version != PG_ABI_VERSION) return fail(PG_E_INVALID, "image: ABI version %u != %u", h.abi_version, PG_ABI_VERSION);
  if (h.image_bytes != n) return fail(PG_E_INVALID, "image: header says %llu bytes, buffer has %llu",
                                      (unsigned long long)h.image_bytes, (unsigned long long)n);
  // [off, off + count * size) inside the buffer, aligned; an empty array may carry any offset (it is never read)
  auto span = [&](uint64_t off, uint64_t count, uint64_t size, uint64_t align, const char* what) -> const void* {
    if (!count) return nullptr;
    uint64_t bytes;
    if (__builtin_mul_overflow(count, size, &bytes) || off < sizeof(pg_image_header) || off % align || off > n ||
        bytes > n - off) {
      fail(PG_E_INVALID, "image: %s (offset %llu, %llu x %llu bytes) outside the %llu-byte buffer or misaligned", what,
           (unsigned long long)off, (unsigned long long)count, (unsigned long long)size, (unsigned long long)n);
      return (const void*)1;  // sentinel: rejected
    }
    return base + off;
  };
  auto bad = [](const void* p) { return p == (const void*)1; };
  if (h.num_segments > (1u << 24) || h.num_leaves > (1u << 16) || h.num_ops > (1u << 20) || h.num_aggs > 64 ||
      h.num_keys > 64 || h.num_order > 64)
    return fail(PG_E_INVALID, "image: counts out of range");
  const pg_image_segment* segs = (const pg_image_segment*)span(h.segments_off, h.num_segments, sizeof(pg_image_segment), 8, "segments");
  const int32_t* ops = (const int32_t*)span(h.ops_off, h.num_ops, 4, 4, "ops");
  const pg_agg* aggs = (const pg_agg*)span(h.aggs_off, h.num_aggs, sizeof(pg_agg), 8, "aggs");
  const pg_key* keys = (const pg_key*)span(h.keys_off, h.num_keys, sizeof(pg_key), 8, "keys");
  const pg_order* order = (const pg_order*)span(h.order_off, h.num_order, sizeof(pg_order), 4, "order");
  if (bad(segs) || bad(ops) || bad(aggs) || bad(keys) || bad(order)) return PG_E_INVALID;
  out.segs.resize(h.num_segments);
  out.leaves.resize((uint64_t)h.num_segments * h.num_leaves);
  for (uint32_t si = 0; si < h.num_segments; si++) {
    const pg_image_segment& is = segs[si];
    const pg_image_leaf* il = (const pg_image_leaf*)span(is.leaves_off, h.num_leaves, sizeof(pg_image_leaf), 8, "leaves");
    if (bad(il)) return PG_E_INVALID;
    pg_leaf* dst = out.leaves.data() + (uint64_t)si * h.num_leaves;
    for (uint32_t li = 0; li < h.num_leaves; li++) {
      const pg_image_leaf& x = il[li];
      pg_leaf& y = dst[li];
      memcpy(&y, &x, sizeof(pg_leaf));  // same layout; the two offsets are replaced below
      y.ids = nullptr;
      y.values = nullptr;
      if (x.ids_off) {
        const void* p = span(x.ids_off, x.num_ids, 4, 4, "leaf ids");
        if (bad(p) || !p) return bad(p) ? PG_E_INVALID : fail(PG_E_INVALID, "image: leaf %u ids_off with num_ids 0", li);
        y.ids = (const int32_t*)p;
      }
      if (x.values_off) {
        const uint64_t nv = x.num_values ? x.num_values : x.num_ids;
        const void* p = span(x.values_off, nv, 8, 8, "leaf values");
        if (bad(p) || !p) return bad(p) ? PG_E_INVALID : fail(PG_E_INVALID, "image: leaf %u values_off with no values", li);
        y.values = p;
      }
    }
    out.segs[si].seg_key = is.seg_key;
    out.segs[si].num_docs = is.num_docs;
    out.segs[si].leaves = dst;
  }
  pg_plan& p = out.plan;
  p.abi_version = h.abi_version;
  p.num_segments = h.num_segments;
  p.segments = out.segs.data();
  p.num_leaves = h.num_leaves;
  p.num_ops = h.num_ops;
  p.ops = ops;
  p.num_aggs = h.num_aggs;
  p.num_keys = h.num_keys;
  p.aggs = aggs;
  p.keys = keys;
  p.num_groups_limit = h.num_groups_limit;
  p.query_id = h.query_id;
  p.deadline_ms = h.deadline_ms;
  p.stream = nullptr;
  p.flags = h.flags;
  p.num_order = h.num_order;
  p.order = order;
  p.limit = h.limit;
  p.trim_threshold = h.trim_threshold;
  return PG_OK;
}


// ------------------------------------------------------------------------------------------ multi-device combine
//
// pg_init_devices binds one process to several logical devices (HIP devices, possibly repeated).  Each logical device
// has one worker thread bound to its GPU, which runs every device call of that logical device (uploads, scans, merges,
// finalisation) with its own stream and per-thread state.  Segments are placed on a logical device at their first
// upload (pg_segment_place, else round-robin).  A query's pg_execute* splits the plan's segments by logical device,
// runs the sub-plans concurrently, and merges the partial states on the first participating device -- the in-process
// form of BaseCombineOperator.mergeResults (operator/combine/BaseCombineOperator.java:190-233) across GPUs:
//   * dense states of one layout: the other devices' state arrays are copied over xGMI (hipMemcpyPeerAsync; a plain
//     device copy when two logical devices share a GPU) and merged element-wise (merge_dense_kernel: SUM, 128-bit
//     SUM, MIN, MAX, OR) -- AggregationFunction.merge of every group at once;
//   * anything else (hash tables, tuple states, mixed modes): every device exports its groups as rows
//     (pg_partials_export), the rows are copied to the merging device and inserted-and-merged into a fresh table
//     (pg_partials_create / pg_partials_merge: IndexedTable.upsert by key).
// The layout choices the merge depends on are made once for the whole plan (global_layout: integer-exact vs
// fixed-point sums and their exponent windows, the dense-vs-hash sizing), so every device's state agrees.
struct TaskResult {
  int rc = PG_OK;
  std::string err;
  pg_timing timing{};
  pg_trace trace{};
};

thread_local bool t_is_worker = false;

struct Worker {
  uint32_t ldev = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::function<void()>> q;
  void loop() {
    t_ldev = (int)ldev;
    t_is_worker = true;
    (void)ensure_device();
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(mu);
        cv.wait(g, [&] { return !q.empty(); });
        f = std::move(q.front());
        q.pop_front();
      }
      f();
    }
  }
};
std::vector<Worker*>* g_workers = nullptr;  // multi-device mode only; the workers live as long as the process

bool multi_device() { return g_workers != nullptr; }
bool on_ldev(uint32_t ldev) { return !multi_device() || (t_is_worker && t_ldev == (int)ldev); }

std::future<TaskResult> post(uint32_t ldev, std::function<int()> fn) {
  auto task = std::make_shared<std::packaged_task<TaskResult()>>([fn = std::move(fn)]() {
    TaskResult r;
    try {
      r.rc = fn();
    } catch (const std::exception& e) {
      r.rc = fail(PG_E_NOMEM, "%s", e.what());
    }
    if (r.rc) r.err = t_err;
    r.timing = t_timing;
    r.trace = t_trace;
    return r;
  });
  std::future<TaskResult> f = task->get_future();
  Worker* w = (*g_workers)[ldev];
  {
    std::lock_guard<std::mutex> g(w->mu);
    w->q.emplace_back([task] { (*task)(); });
  }
  w->cv.notify_one();
  return f;
}

// fn on ldev's worker, synchronously (inline when this thread is that worker); its error message (and with `timing`,
// its timing and trace records) become the calling thread's
int run_on(uint32_t ldev, std::function<int()> fn, bool timing = false) {
  if (on_ldev(ldev)) return fn();
  TaskResult r = post(ldev, std::move(fn)).get();
  if (r.rc) t_err = r.err;
  if (timing) {
    t_timing = r.timing;
    t_trace = r.trace;
  }
  return r.rc;
}

uint32_t partial_ldev(const pg_partials* p) { return p && p->impl ? ((const PartialsImpl*)p->impl)->ldev : 0u; }

std::mutex g_place_mu;
std::unordered_map<uint64_t, uint32_t> g_place;  // seg_key -> logical device (multi-device mode)
uint32_t g_place_next = 0;

// The logical device of a segment: where it is resident, else its placement (pg_segment_place), else the next one
// round-robin in first-upload order
uint32_t placement(uint64_t seg_key) {
  {
    std::shared_lock<std::shared_mutex> lk(g_seg_mu);
    auto it = g_segs.find(seg_key);
    if (it != g_segs.end()) return it->second->ldev;
  }
  std::lock_guard<std::mutex> g(g_place_mu);
  auto it = g_place.find(seg_key);
  if (it != g_place.end()) return it->second;
  const uint32_t d = g_place_next++ % (uint32_t)std::max<size_t>(1, g_ldev_phys.size());
  g_place.emplace(seg_key, d);
  return d;
}

// The layout choices every logical device's partial state must share (under g_seg_mu, shared): per SUM / AVG
// aggregation integer-exact or fixed point over the WHOLE plan's segments and docs, and the fixed-point windows from
// the table-wide bounds of every segment (unless the caller gave them: PG_SUM_BOUNDS).
int global_layout(const pg_plan* plan, std::vector<pg_agg>& aggs, LayoutHint& hint) {
  hint.on = true;
  hint.docs = 0;
  hint.integer = 0;
  for (uint32_t si = 0; si < plan->num_segments; si++) hint.docs += plan->segments[si].num_docs;
  for (uint32_t a = 0; a < plan->num_aggs; a++) {
    pg_agg& g = aggs[a];
    if (g.fn != PG_AGG_SUM && g.fn != PG_AGG_AVG) continue;
    const bool two = g.op != PG_EXPR_COL;
    SumBounds sb;
    uint64_t mv_vals = 0;
    for (uint32_t si = 0; si < plan->num_segments; si++) {
      auto it = g_segs.find(plan->segments[si].seg_key);
      if (it == g_segs.end()) return fail(PG_E_NOTFOUND, "segment %llu not resident", (unsigned long long)plan->segments[si].seg_key);
      auto ca = it->second->cols.find(g.col_a);
      auto cb = two ? it->second->cols.find(g.col_b) : it->second->cols.end();
      if (ca == it->second->cols.end() || (two && cb == it->second->cols.end()))
        continue;  // the device's own compile reports the missing column
      if (ca->second.dtype > PG_DOUBLE || (two && cb->second.dtype > PG_DOUBLE)) continue;
      sum_bounds_add(sb, &ca->second, two ? &cb->second : nullptr);
      mv_vals += ca->second.num_values;
    }
    if (sum_as_int(sb, g, two, plan->flags, (g.flags & PG_AGG_MV_VALUES) ? mv_vals : hint.docs)) {
      hint.integer |= 1u << a;
      continue;
    }
    int klo, khi;
    bool nonfinite, any;
    sum_windows(sb, g, two, klo, khi, nonfinite, any);
    if (!(g.sum_flags & PG_SUM_BOUNDS)) {
      g.sum_exp = khi;
      g.sum_exp_lo = klo;
      g.sum_flags |= PG_SUM_BOUNDS;
    }
    if (nonfinite) g.sum_flags |= PG_SUM_NONFINITE;
  }
  return PG_OK;
}

// Copy n bytes of device memory between logical devices (an xGMI peer copy between two GPUs)
hipError_t copy_between(void* dst, uint32_t dst_ldev, const void* src, uint32_t src_ldev, uint64_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  const int dd = g_ldev_phys[dst_ldev], sd = g_ldev_phys[src_ldev];
  if (dd == sd) return hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToDevice, s);
  return hipMemcpyPeerAsync(dst, dd, src, sd, n, s);
}

// Merge the dense states `others` into `T` (all of one layout), on T's logical device.
int merge_dense_into(PartialsImpl* T, const std::vector<PartialsImpl*>& others) {
  hipStream_t s = thread_stream();
  Partials& P = T->P;
  const uint64_t G = P.num_slots;
  const uint64_t bytes[5] = {G * 8ull * P.n_i64, G * 16ull * P.n_fx, G * 8ull * P.n_min, G * 8ull * P.n_max,
                             G * 4ull * P.bit_words};
  for (PartialsImpl* O : others) {
    const Partials& S = O->P;
    StateView sv = S.view();
    DevBuf tmp[5];
    if (g_ldev_phys[O->ldev] != g_ldev_phys[T->ldev]) {  // another GPU: bring its arrays here first
      void* src[5] = {S.i64.p, S.fx.p, S.mn.p, S.mx.p, S.bits.p};
      void** dst[5] = {(void**)&sv.i64, (void**)&sv.fx, (void**)&sv.mn, (void**)&sv.mx, (void**)&sv.bits};
      for (int i = 0; i < 5; i++) {
        if (!bytes[i]) continue;
        int rc = tmp[i].alloc_pooled(bytes[i]);
        if (rc) return rc;
        HIP_CHECK(copy_between(tmp[i].p, T->ldev, src[i], O->ldev, bytes[i], s));
        *dst[i] = tmp[i].p;
      }
    }
    HIP_CHECK(launch_merge_dense(P.view(), sv, s));
    HIP_CHECK(hipStreamSynchronize(s));
    P.flags |= S.flags & PG_RESULT_GROUPS_LIMIT_REACHED;
  }
  return PG_OK;
}

bool same_dense_layout(const std::vector<pg_partials*>& ps) {
  for (const pg_partials* p : ps)
    if (p->mode != PG_STATE_DENSE || p->num_slots != ps[0]->num_slots || p->n_i64 != ps[0]->n_i64 ||
        p->n_fx != ps[0]->n_fx || p->n_min != ps[0]->n_min || p->n_max != ps[0]->n_max ||
        p->bitmap_words != ps[0]->bitmap_words || ((const PartialsImpl*)p->impl)->P.wide)
      return false;
  return true;
}

int free_partials_everywhere(std::vector<pg_partials*>& ps) {
  for (pg_partials*& p : ps)
    if (p) { (void)pg_partials_free(p); p = nullptr; }
  return PG_OK;
}

// The in-library combine of the partial states ps (one per participating logical device, ps[0] on the merging
// device): the merged state, on ps[0]'s device; consumes ps.
int merge_partials_multi(std::vector<pg_partials*>& ps, pg_partials** out) {
  for (const pg_partials* p : ps)
    if (p->layout != ps[0]->layout || p->fx_sig != ps[0]->fx_sig || p->row_bytes != ps[0]->row_bytes) {
      free_partials_everywhere(ps);
      return fail(PG_E_INVALID, "partial state layouts differ between logical devices");
    }
  pg_stats st{};
  uint32_t flags = 0;
  for (const pg_partials* p : ps) {
    st.num_docs_scanned += p->stats.num_docs_scanned;
    st.num_entries_scanned_in_filter += p->stats.num_entries_scanned_in_filter;
    st.num_entries_scanned_post_filter += p->stats.num_entries_scanned_post_filter;
    st.num_total_docs += p->stats.num_total_docs;
    st.num_segments_processed += p->stats.num_segments_processed;
    st.num_segments_matched += p->stats.num_segments_matched;
    flags |= p->flags & PG_RESULT_GROUPS_LIMIT_REACHED;
  }
  const uint32_t d0 = partial_ldev(ps[0]);
  int rc;
  if (same_dense_layout(ps)) {
    std::vector<PartialsImpl*> others;
    for (size_t i = 1; i < ps.size(); i++) others.push_back((PartialsImpl*)ps[i]->impl);
    rc = run_on(d0, [&] { return merge_dense_into((PartialsImpl*)ps[0]->impl, others); });
    pg_partials* m = ps[0];
    ps[0] = nullptr;
    free_partials_everywhere(ps);
    if (rc) { (void)pg_partials_free(m); return rc; }
    m->stats = st;
    m->flags = flags;
    *out = m;
    return PG_OK;
  }
  // the row exchange: every device exports its groups (on its own worker, concurrently), the merging device inserts
  // them into a fresh table
  const uint64_t rb = ps[0]->row_bytes;
  std::vector<DevBuf> rows(ps.size());
  std::vector<uint64_t> nrows(ps.size(), 0);
  std::vector<std::future<TaskResult>> fut;
  for (size_t i = 0; i < ps.size(); i++) {
    fut.push_back(post(partial_ldev(ps[i]), [&, i] {
      uint64_t n = 0;
      int r = pg_partials_export(ps[i], 1, nullptr, 0, &n, nullptr);
      if (r) return r;
      if ((r = rows[i].alloc_pooled(n * rb + 8))) return r;
      nrows[i] = n;
      return n ? pg_partials_export(ps[i], 1, rows[i].p, n, &n, nullptr) : PG_OK;
    }));
  }
  rc = PG_OK;
  for (auto& f : fut) {
    TaskResult r = f.get();
    if (r.rc && !rc) { rc = r.rc; t_err = r.err; }
  }
  pg_partials* m = nullptr;
  if (!rc) {
    uint64_t total = 0;
    for (uint64_t n : nrows) total += n;
    rc = run_on(d0, [&] {
      int r = pg_partials_create(ps[0], std::max<uint64_t>(total, 1), &m);
      if (r) return r;
      hipStream_t s = thread_stream();
      for (size_t i = 0; i < ps.size() && !r; i++) {
        if (!nrows[i]) continue;
        const uint32_t src = partial_ldev(ps[i]);
        const void* at = rows[i].p;
        DevBuf tmp;
        if (g_ldev_phys[src] != g_ldev_phys[d0]) {
          if ((r = tmp.alloc_pooled(nrows[i] * rb + 8))) break;
          if (copy_between(tmp.p, d0, rows[i].p, src, nrows[i] * rb, s) != hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess) {
            r = fail(PG_E_HIP, "row copy between logical devices %u and %u failed", src, d0);
            break;
          }
          at = tmp.p;
        }
        r = pg_partials_merge(m, at, nrows[i], nullptr);
      }
      return r;
    });
  }
  rows.clear();
  free_partials_everywhere(ps);
  if (rc) {
    if (m) (void)pg_partials_free(m);
    return rc;
  }
  m->stats = st;
  m->flags = flags;
  *out = m;
  return PG_OK;
}

// pg_execute_partial in multi-device mode: the plan's segments split by logical device, one sub-plan per device with
// segments run concurrently, their states merged (merge_partials_multi).
int execute_partial_multi(const pg_plan* plan, pg_partials** out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  *out = nullptr;
  if (!plan) return fail(PG_E_INVALID, "null plan");
  if (plan->abi_version != PG_ABI_VERSION)
    return fail(PG_E_INVALID, "plan ABI version %u, library %d", plan->abi_version, PG_ABI_VERSION);
  if (plan->num_segments && !plan->segments) return fail(PG_E_INVALID, "null segment list");
  if (plan->num_aggs && !plan->aggs) return fail(PG_E_INVALID, "null aggregation list");
  if (plan->num_aggs > (uint32_t)kMaxAggs) return fail(PG_E_UNSUPPORTED, "more than %d aggregations", kMaxAggs);
  const double t0 = wall_ms();
  const uint32_t N = (uint32_t)g_ldev_phys.size();
  struct Sub {
    std::vector<pg_segment_ref> segs;
    pg_plan plan;
    pg_partials* out = nullptr;
  };
  std::vector<Sub> sub(N);
  std::vector<pg_agg> aggs(plan->aggs, plan->aggs + plan->num_aggs);
  LayoutHint hint;
  {
    std::shared_lock<std::shared_mutex> lk(g_seg_mu);
    for (uint32_t si = 0; si < plan->num_segments; si++) {
      auto it = g_segs.find(plan->segments[si].seg_key);
      if (it == g_segs.end())
        return fail(PG_E_NOTFOUND, "segment %llu not resident", (unsigned long long)plan->segments[si].seg_key);
      sub[it->second->ldev].segs.push_back(plan->segments[si]);
    }
    const int rc = global_layout(plan, aggs, hint);
    if (rc) return rc;
  }
  std::vector<uint32_t> run;
  for (uint32_t d = 0; d < N; d++)
    if (!sub[d].segs.empty()) run.push_back(d);
  if (run.empty()) run.push_back(0);
  std::vector<std::future<TaskResult>> fut;
  for (uint32_t d : run) {
    Sub& x = sub[d];
    x.plan = *plan;
    x.plan.num_segments = (uint32_t)x.segs.size();
    x.plan.segments = x.segs.empty() ? nullptr : x.segs.data();
    x.plan.aggs = aggs.empty() ? nullptr : aggs.data();
    x.plan.stream = nullptr;  // the caller's stream belongs to its own device: each worker uses its own
    fut.push_back(post(d, [&x, &hint] {
      t_layout = hint;
      const int r = pg_execute_partial(&x.plan, &x.out);
      t_layout = LayoutHint{};
      return r;
    }));
  }
  int rc = PG_OK;
  pg_timing tm{};
  pg_trace tr{};
  uint64_t matched = 0;
  for (size_t i = 0; i < fut.size(); i++) {
    TaskResult r = fut[i].get();
    if (r.rc && !rc) { rc = r.rc; t_err = r.err; }
    if (i == 0) { tm = r.timing; tr = r.trace; }
    tm.scan_ms = std::max(tm.scan_ms, r.timing.scan_ms);
    tm.prepass_ms = std::max(tm.prepass_ms, r.timing.prepass_ms);
    tr.path |= r.trace.path;
    matched += r.trace.num_docs_matched;
  }
  std::vector<pg_partials*> ps;
  for (uint32_t d : run)
    if (sub[d].out) ps.push_back(sub[d].out);
  if (rc) {
    free_partials_everywhere(ps);
    return rc;
  }
  if (ps.size() == 1) {
    *out = ps[0];
  } else if ((rc = merge_partials_multi(ps, out))) {
    return rc;
  }
  tm.execute_wall_ms = (float)(wall_ms() - t0);
  tr.num_docs_matched = matched;
  tr.num_segments = plan->num_segments;
  tr.wall_ms = tm.execute_wall_ms;
  t_timing = tm;
  t_trace = tr;
  return PG_OK;
}

// pg_dict_id_sets over segments resident on several logical devices: each device looks up its own segments
int dict_id_sets_multi(const uint64_t* seg_keys, uint32_t num_segments, uint32_t col_id, uint32_t data_type,
                       const void* values, uint32_t num_values, int32_t* out_ids, uint32_t* out_counts) {
  const uint32_t N = (uint32_t)g_ldev_phys.size();
  std::vector<std::vector<uint32_t>> idx(N);
  for (uint32_t si = 0; si < num_segments; si++) idx[placement(seg_keys[si])].push_back(si);
  for (uint32_t d = 0; d < N; d++) {
    if (idx[d].empty()) continue;
    std::vector<uint64_t> keys(idx[d].size());
    for (size_t i = 0; i < keys.size(); i++) keys[i] = seg_keys[idx[d][i]];
    std::vector<int32_t> ids((uint64_t)keys.size() * num_values);
    std::vector<uint32_t> cnt(keys.size());
    const int rc = run_on(d, [&] {
      return pg_dict_id_sets(keys.data(), (uint32_t)keys.size(), col_id, data_type, values, num_values, ids.data(),
                             cnt.data());
    });
    if (rc) return rc;
    for (size_t i = 0; i < keys.size(); i++) {
      memcpy(out_ids + (uint64_t)idx[d][i] * num_values, ids.data() + i * (uint64_t)num_values, 4ull * num_values);
      out_counts[idx[d][i]] = cnt[i];
    }
  }
  return PG_OK;
}

}  // namespace

// ============================================================================================ C ABI

extern "C" {

int pg_abi_version(void) { return PG_ABI_VERSION; }

// PG_SEGV_TRACE=1: a host SIGSEGV prints the native frames (library offsets for addr2line) before the default action
static void segv_trace(int sig) {
  void* fr[64];
  const int n = backtrace(fr, 64);
  const char msg[] = "libpinot_gpu: fatal signal, native frames:\n";
  (void)!write(2, msg, sizeof(msg) - 1);
  backtrace_symbols_fd(fr, n, 2);
  signal(sig, SIG_DFL);
  raise(sig);
}

int pg_init_devices(const int* devices, uint32_t n) {
  std::lock_guard<std::mutex> g(g_init_mu);
  if (getenv("PG_SEGV_TRACE") && atoi(getenv("PG_SEGV_TRACE"))) signal(SIGSEGV, segv_trace);
  if (!devices || n == 0 || n > 64) return fail(PG_E_INVALID, "device list of %u entries", n);
  int vis = 0;
  if (hipGetDeviceCount(&vis) != hipSuccess || vis == 0) return fail(PG_E_HIP, "no HIP device visible");
  for (uint32_t i = 0; i < n; i++)
    if (devices[i] < 0 || devices[i] >= vis || devices[i] >= kMaxPhys)
      return fail(PG_E_INVALID, "device %d out of range (%d visible)", devices[i], vis);
  if (g_device >= 0) {  // idempotent for the same binding
    if (g_ldev_phys.size() == n && std::equal(g_ldev_phys.begin(), g_ldev_phys.end(), devices)) return PG_OK;
    return fail(PG_E_STATE, "already bound to device %d (%zu logical devices)", g_device, g_ldev_phys.size());
  }
  for (uint32_t i = 0; i < n; i++) {  // xGMI peer access between the distinct GPUs (copies work without it, staged)
    for (uint32_t j = 0; j < n; j++) {
      if (devices[i] == devices[j]) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, devices[i], devices[j]) == hipSuccess && can && hipSetDevice(devices[i]) == hipSuccess) {
        const hipError_t e = hipDeviceEnablePeerAccess(devices[j], 0);
        if (e != hipSuccess) (void)hipGetLastError();  // already enabled (another pair entry) is fine
      }
    }
  }
  HIP_CHECK(hipSetDevice(devices[0]));
  g_ldev_phys.assign(devices, devices + n);
  g_device = devices[0];
  init_grid_caps();
  int rc = init_cancel_flags();
  if (rc) return rc;
  if (n > 1) {
    auto* ws = new std::vector<Worker*>();
    for (uint32_t i = 0; i < n; i++) {
      Worker* w = new Worker();
      w->ldev = i;
      ws->push_back(w);
      std::thread([w] { w->loop(); }).detach();
    }
    g_workers = ws;
  }
  return PG_OK;
}

int pg_init(int device) { return pg_init_devices(&device, 1); }

int pg_num_devices(uint32_t* out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  *out = (uint32_t)g_ldev_phys.size();
  return g_device < 0 ? fail(PG_E_STATE, "pg_init has not been called") : PG_OK;
}

int pg_segment_place(uint64_t seg_key, uint32_t ldev) {
  if (g_device < 0) return fail(PG_E_STATE, "pg_init has not been called");
  if (ldev >= g_ldev_phys.size()) return fail(PG_E_INVALID, "logical device %u of %zu", ldev, g_ldev_phys.size());
  {
    std::shared_lock<std::shared_mutex> lk(g_seg_mu);
    auto it = g_segs.find(seg_key);
    if (it != g_segs.end() && it->second->ldev != ldev)
      return fail(PG_E_STATE, "segment %llu is resident on logical device %u (release it first)",
                  (unsigned long long)seg_key, it->second->ldev);
  }
  std::lock_guard<std::mutex> g(g_place_mu);
  g_place[seg_key] = ldev;
  return PG_OK;
}

int pg_segment_device(uint64_t seg_key, uint32_t* ldev) {
  if (!ldev) return fail(PG_E_INVALID, "null out");
  std::shared_lock<std::shared_mutex> lk(g_seg_mu);
  auto it = g_segs.find(seg_key);
  if (it == g_segs.end()) return fail(PG_E_NOTFOUND, "segment %llu not resident", (unsigned long long)seg_key);
  *ldev = it->second->ldev;
  return PG_OK;
}

int pg_last_error(char* buf, size_t n) {
  if (buf && n) {
    strncpy(buf, t_err.c_str(), n - 1);
    buf[n - 1] = 0;
  }
  return (int)t_err.size();
}

int pg_resident_bytes(uint64_t* out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  std::shared_lock<std::shared_mutex> lk(g_seg_mu);
  uint64_t t = 0;
  for (auto& kv : g_segs)
    for (auto& c : kv.second->cols)
      t += c.second.dict.bytes + c.second.words.bytes + c.second.mv_offsets.bytes + c.second.mv_cnt.bytes + c.second.roaring.bytes +
           c.second.containers.bytes + c.second.inv_keydir.bytes + c.second.keymap.bytes + c.second.vals.bytes + c.second.rawv.bytes;
  *out = t;
  return PG_OK;
}

int pg_cancel(uint64_t query_id) {
  std::lock_guard<std::mutex> g(g_cancel_mu);
  g_cancelled.insert(query_id);
  auto r = g_inflight.equal_range(query_id);
  for (auto it = r.first; it != r.second; ++it) g_flags[it->second] = 1u;  // running launches stop at their next tile
  return PG_OK;
}

int pg_column_upload(uint64_t seg_key, uint32_t col_id, const pg_col_desc* desc, const void* src, uint64_t nbytes) {
  if (multi_device() && !t_is_worker) {
    const uint32_t d = placement(seg_key);
    return run_on(d, [=] { return pg_column_upload(seg_key, col_id, desc, src, nbytes); });
  }
  int rc = ensure_device();
  if (rc) return rc;
  if (!desc || (!src && nbytes)) return fail(PG_E_INVALID, "null descriptor or source");
  try {
    return upload_column(seg_key, col_id, desc, src, nbytes);
  } catch (const std::exception& e) {
    return fail(PG_E_NOMEM, "upload failed: %s", e.what());
  }
}

int pg_segment_release(uint64_t seg_key) {
  if (multi_device() && !t_is_worker) {
    const uint32_t d = placement(seg_key);
    const int r = run_on(d, [=] { return pg_segment_release(seg_key); });
    std::lock_guard<std::mutex> g(g_place_mu);
    g_place.erase(seg_key);
    return r;
  }
  int rc = ensure_device();
  if (rc) return rc;
  std::unique_lock<std::shared_mutex> lk(g_seg_mu);
  auto it = g_segs.find(seg_key);
  if (it == g_segs.end()) return fail(PG_E_NOTFOUND, "segment %llu not resident", (unsigned long long)seg_key);
  delete it->second;
  g_segs.erase(it);
  return PG_OK;
}

int pg_execute_partial(const pg_plan* plan, pg_partials** out) {
  if (multi_device() && !t_is_worker) return execute_partial_multi(plan, out);
  int rc = ensure_device();
  if (rc) return rc;
  if (!out) return fail(PG_E_INVALID, "null out");
  *out = nullptr;
  PartialsImpl* impl = new (std::nothrow) PartialsImpl();
  if (!impl) return fail(PG_E_NOMEM, "out of host memory");
  impl->ldev = (uint32_t)t_ldev;
  pg_stats st;
  const double t0 = wall_ms();
  t_timing.host_compile_ms = 0;
  t_timing.finalize_wall_ms = 0;
  memset(&t_trace, 0, sizeof(t_trace));
  t_trace.query_id = plan ? plan->query_id : 0;
  t_trace.stream_leaf = 0xFFFFFFFFu;
  try {
    rc = plan_needs_wide(plan) ? run_wide(plan, impl->P, st) : run_with_retries(plan, impl->P, st);
    t_timing.execute_wall_ms = (float)(wall_ms() - t0);
  } catch (const std::exception& e) {
    rc = fail(PG_E_NOMEM, "execute failed: %s", e.what());
  }
  t_trace.num_docs_matched = rc ? 0 : st.num_docs_scanned;
  t_trace.wall_ms = (float)(wall_ms() - t0);
  if (rc) { delete impl; return rc; }
  pg_partials* p = (pg_partials*)calloc(1, sizeof(pg_partials));
  if (!p) { delete impl; return fail(PG_E_NOMEM, "out of host memory"); }
  p->stats = st;
  fill_handle(p, impl);
  *out = p;
  return PG_OK;
}

int pg_partials_finalize(pg_partials* p, const pg_plan* plan, pg_result** out) {
  if (!on_ldev(partial_ldev(p))) return run_on(partial_ldev(p), [=] { return pg_partials_finalize(p, plan, out); }, true);
  int rc = ensure_device();
  if (rc) return rc;
  if (!p || !plan || !out || !p->impl) return fail(PG_E_INVALID, "null argument");
  try {
    return finalize(p, plan, out);
  } catch (const std::exception& e) {
    return fail(PG_E_NOMEM, "finalize failed: %s", e.what());
  }
}

int pg_partials_free(pg_partials* p) {
  if (!p) return PG_OK;
  if (!on_ldev(partial_ldev(p))) return run_on(partial_ldev(p), [=] { return pg_partials_free(p); });
  ensure_device();
  delete (PartialsImpl*)p->impl;
  free(p);
  return PG_OK;
}

int pg_partials_copy(pg_partials* p, int dir, void* i64, void* fx, void* mn, void* mx, void* stream) {
  if (!on_ldev(partial_ldev(p)))
    return run_on(partial_ldev(p), [=] { return pg_partials_copy(p, dir, i64, fx, mn, mx, nullptr); });
  int rc = ensure_device();
  if (rc) return rc;
  if (!p || !p->impl || (dir != PG_COPY_OUT && dir != PG_COPY_IN)) return fail(PG_E_INVALID, "bad partials / direction");
  if (p->mode != PG_STATE_DENSE) return fail(PG_E_INVALID, "pg_partials_copy needs a dense state (use pg_partials_export)");
  if (((PartialsImpl*)p->impl)->P.wide)
    return fail(PG_E_UNSUPPORTED, "wide group keys are tuple slots local to one state: no cross-state merge");
  hipStream_t s = stream ? (hipStream_t)stream : thread_stream();
  void* mine[4] = {p->i64, p->fx, p->mn, p->mx};
  void* theirs[4] = {i64, fx, mn, mx};
  const uint64_t bytes[4] = {p->num_slots * 8ull * p->n_i64, p->num_slots * 16ull * p->n_fx,
                             p->num_slots * 8ull * p->n_min, p->num_slots * 8ull * p->n_max};
  if (fx && p->n_fx)  // the exact sums travel as 32-bit limbs (4 per sum): a word-wise SUM merges those
    HIP_CHECK(launch_fx_limbs((unsigned long long*)p->fx, (long long*)fx, p->num_slots * p->n_fx, dir == PG_COPY_IN, s));
  for (int i = 0; i < 4; i++) {
    if (i == 1 || !theirs[i] || !bytes[i]) continue;
    if (dir == PG_COPY_OUT) HIP_CHECK(hipMemcpyAsync(theirs[i], mine[i], bytes[i], hipMemcpyDeviceToDevice, s));
    else HIP_CHECK(hipMemcpyAsync(mine[i], theirs[i], bytes[i], hipMemcpyDeviceToDevice, s));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  return PG_OK;
}

// Wide keys (the state's packed keys are slots of its own tuple table): rows { state row | tuple }, the owner part from
// the tuple (table-global key ids), so the same group goes to the same owner from every GPU.
int export_wide(Partials& P, uint32_t num_parts, void* dst, uint64_t dst_rows, uint64_t* part_counts, hipStream_t s) {
  const WideKeys& W = *P.wide;
  Scratch sc(s);
  int rc = PG_OK;
  const StateView v = P.view();
  const size_t tb = select_temp_bytes(P.num_slots);
  uint32_t* slots = sc.get<uint32_t>(P.num_slots, rc);
  uint32_t* d_num = sc.get<uint32_t>(2, rc);
  void* temp = sc.get<uint8_t>(tb, rc);
  if (rc) return rc;
  HIP_CHECK(launch_select_slots(v, SEL_PRESENT, 0, 1, slots, d_num, temp, tb, s));
  uint32_t n = 0;
  if ((rc = read_back(d_num, n, s))) return rc;
  const uint64_t rb = row_bytes(v), rbw = rb + wide_tuple_bytes(W.K);
  uint32_t* owner = sc.get<uint32_t>((uint64_t)n + 1, rc);
  uint8_t* rows = sc.get<uint8_t>(rb * n + 8, rc);
  if (rc) return rc;
  // the rows (key word = tuple slot: a hash state's key, a dense state's slot), their owners from the tuples
  HIP_CHECK(launch_gather_rows(v, slots, n, 1, rows, s));
  HIP_CHECK(launch_wide_owner((const uint32_t*)W.tuples.p, W.K, rows, rb, n, num_parts, owner, s));
  std::vector<uint32_t> own(n), sl(n);
  if (n) {
    HIP_CHECK(hipMemcpyAsync(own.data(), owner, 4ull * n, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipMemcpyAsync(sl.data(), slots, 4ull * n, hipMemcpyDeviceToHost, s));
  }
  HIP_CHECK(hipStreamSynchronize(s));
  std::vector<uint64_t> at(num_parts + 1, 0);
  for (uint32_t i = 0; i < n; i++) at[own[i] + 1]++;
  for (uint32_t q = 0; q < num_parts; q++) part_counts[q] = at[q + 1];
  if (!dst) return PG_OK;
  if (n > dst_rows) return fail(PG_E_INVALID, "export buffer of %llu rows too small", (unsigned long long)dst_rows);
  for (uint32_t q = 0; q < num_parts; q++) at[q + 1] += at[q];
  std::vector<uint32_t> order(n);  // state slots bucketed by owner part, stable
  for (uint32_t i = 0; i < n; i++) order[at[own[i]]++] = sl[i];
  if (n) HIP_CHECK(hipMemcpyAsync(slots, order.data(), 4ull * n, hipMemcpyHostToDevice, s));
  HIP_CHECK(launch_gather_rows(v, slots, n, 1, rows, s));
  HIP_CHECK(launch_widen_rows(rows, rb, (const uint32_t*)W.tuples.p, W.K, n, (uint8_t*)dst, rbw, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return PG_OK;
}

int pg_partials_export(pg_partials* p, uint32_t num_parts, void* dst, uint64_t dst_rows, uint64_t* part_counts,
                       void* stream) {
  if (!on_ldev(partial_ldev(p)))
    return run_on(partial_ldev(p), [=] { return pg_partials_export(p, num_parts, dst, dst_rows, part_counts, nullptr); });
  int rc = ensure_device();
  if (rc) return rc;
  if (!p || !p->impl || !num_parts || !part_counts) return fail(PG_E_INVALID, "bad export arguments");
  try {
    Partials& P = ((PartialsImpl*)p->impl)->P;
    hipStream_t s = stream ? (hipStream_t)stream : thread_stream();
    if (P.wide) return export_wide(P, num_parts, dst, dst_rows, part_counts, s);
    Scratch sc(s);
    const StateView v = P.view();
    const size_t tb = select_temp_bytes(P.num_slots);
    uint32_t* slots = sc.get<uint32_t>(P.num_slots, rc);
    uint32_t* d_num = sc.get<uint32_t>(2, rc);
    void* temp = sc.get<uint8_t>(tb, rc);
    if (rc) return rc;
    uint64_t at = 0;
    for (uint32_t part = 0; part < num_parts; part++) {
      HIP_CHECK(launch_select_slots(v, SEL_PRESENT_PART, part, num_parts, slots, d_num, temp, tb, s));
      uint32_t n = 0;
      if ((rc = read_back(d_num, n, s))) return rc;
      part_counts[part] = n;
      if (dst) {
        if (at + n > dst_rows) return fail(PG_E_INVALID, "export buffer of %llu rows too small", (unsigned long long)dst_rows);
        HIP_CHECK(launch_gather_rows(v, slots, n, 1, (uint8_t*)dst + at * p->row_bytes, s));
      }
      at += n;
    }
    HIP_CHECK(hipStreamSynchronize(s));
    return PG_OK;
  } catch (const std::exception& e) {
    return fail(PG_E_NOMEM, "export failed: %s", e.what());
  }
}

int pg_partials_create(const pg_partials* like, uint64_t capacity, pg_partials** out) {
  if (!on_ldev(partial_ldev(like)))
    return run_on(partial_ldev(like), [=] { return pg_partials_create(like, capacity, out); });
  int rc = ensure_device();
  if (rc) return rc;
  if (!like || !like->impl || !out) return fail(PG_E_INVALID, "null argument");
  *out = nullptr;
  PartialsImpl* impl = new (std::nothrow) PartialsImpl();
  if (!impl) return fail(PG_E_NOMEM, "out of host memory");
  impl->ldev = (uint32_t)t_ldev;
  try {
    hipStream_t s = thread_stream();
    const Partials& L = ((PartialsImpl*)like->impl)->P;
    rc = hash_like(L, capacity, impl->P, s);
    if (!rc && L.wide) {  // a wide-key merge target: a fresh tuple table; its slots are the hash state's one key
      auto W = std::make_shared<WideKeys>();
      W->K = L.wide->K;
      W->cap = pow2_at_least(std::max<uint64_t>(1024, 2 * capacity));
      if (W->cap > (1ull << 31) || W->cap * (8ull + 4ull * W->K) > kStateBudget) {
        rc = fail(PG_E_UNSUPPORTED, "tuple table of %llu slots exceeds the state budget", (unsigned long long)W->cap);
      } else if (!(rc = W->tags.alloc(W->cap * 8)) && !(rc = W->tuples.alloc(W->cap * 4ull * W->K)) &&
                 !(rc = W->misc.alloc(16))) {
        HIP_CHECK(hipMemsetAsync(W->tags.p, 0, W->cap * 8, s));
        HIP_CHECK(hipMemsetAsync(W->misc.p, 0, 16, s));
        W->key1 = L.wide->key1;
        W->key1.cardinality = (uint32_t)W->cap;
        impl->P.key_card.assign(1, (uint32_t)W->cap);
        impl->P.key_stride.assign(1, 1);
        impl->P.wide = W;
      }
    }
    if (!rc && hipStreamSynchronize(s) != hipSuccess) rc = fail(PG_E_HIP, "state initialisation failed");
  } catch (const std::exception& e) {
    rc = fail(PG_E_NOMEM, "create failed: %s", e.what());
  }
  if (rc) { delete impl; return rc; }
  pg_partials* p = (pg_partials*)calloc(1, sizeof(pg_partials));
  if (!p) { delete impl; return fail(PG_E_NOMEM, "out of host memory"); }
  fill_handle(p, impl);
  *out = p;
  return PG_OK;
}

int pg_partials_merge(pg_partials* p, const void* rows, uint64_t n, void* stream) {
  if (!on_ldev(partial_ldev(p))) return run_on(partial_ldev(p), [=] { return pg_partials_merge(p, rows, n, nullptr); });
  int rc = ensure_device();
  if (rc) return rc;
  if (!p || !p->impl || (!rows && n)) return fail(PG_E_INVALID, "null argument");
  Partials& P = ((PartialsImpl*)p->impl)->P;
  if (P.mode != GM_HASH) return fail(PG_E_INVALID, "pg_partials_merge needs a hash state (pg_partials_create)");
  hipStream_t s = stream ? (hipStream_t)stream : thread_stream();
  const void* merged = rows;
  Scratch sc(s);
  if (P.wide) {  // wide keys: re-intern each row's tuple here, then merge the rows keyed by this table's slots
    WideKeys& W = *P.wide;
    if (!W.tags.p) return fail(PG_E_INVALID, "pg_partials_merge needs a merge target (pg_partials_create)");
    const uint64_t rb = row_bytes(P.view());
    uint8_t* keyed = sc.get<uint8_t>(rb * n + 8, rc);
    if (rc) return rc;
    WideSpec ws;
    memset(&ws, 0, sizeof(ws));
    ws.K = W.K;
    ws.max_fill = (uint32_t)(W.cap / 4 * 3);
    ws.mask = W.cap - 1;
    ws.tags = (unsigned long long*)W.tags.p;
    ws.tuples = (uint32_t*)W.tuples.p;
    ws.fill = (unsigned int*)W.misc.p;
    ws.err = (unsigned int*)W.misc.p + 1;
    HIP_CHECK(launch_intern_rows(ws, (const uint8_t*)rows, n, rb, rb + wide_tuple_bytes(W.K), keyed, s));
    uint32_t we[2] = {0, 0};
    HIP_CHECK(hipMemcpyAsync(we, W.misc.p, 8, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    if (we[1]) return fail(PG_E_NOMEM, "merge tuple table of %llu slots is full", (unsigned long long)W.cap);
    merged = keyed;
  }
  HIP_CHECK(launch_merge_rows(P.view(), (const uint8_t*)merged, n, s));
  uint32_t fe[2] = {0, 0};
  HIP_CHECK(hipMemcpyAsync(fe, P.misc.p, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (fe[1]) return fail(PG_E_NOMEM, "merge table of %llu slots is full", (unsigned long long)P.num_slots);
  return PG_OK;
}

int pg_dict_id_sets(const uint64_t* seg_keys, uint32_t num_segments, uint32_t col_id, uint32_t data_type,
                    const void* values, uint32_t num_values, int32_t* out_ids, uint32_t* out_counts) {
  if (multi_device() && !t_is_worker && g_device >= 0) {
    if ((!seg_keys && num_segments) || (!values && num_values) || (!out_ids && num_segments && num_values) ||
        (!out_counts && num_segments))
      return fail(PG_E_INVALID, "null argument");
    return dict_id_sets_multi(seg_keys, num_segments, col_id, data_type, values, num_values, out_ids, out_counts);
  }
  int rc = ensure_device();
  if (rc) return rc;
  if ((!seg_keys && num_segments) || (!values && num_values) || (!out_ids && num_segments && num_values) ||
      (!out_counts && num_segments))
    return fail(PG_E_INVALID, "null argument");
  if (data_type > PG_DOUBLE) return fail(PG_E_UNSUPPORTED, "dictIds of %u-typed literals", data_type);
  const uint64_t S = num_segments, n = num_values;
  if (!S) return PG_OK;
  if (!n) { memset(out_counts, 0, 4 * S); return PG_OK; }
  try {
    std::vector<DictLookupJob> jobs(S);
    // held until the lookup kernel has finished reading the dictionaries (a concurrent pg_segment_release frees them)
    std::shared_lock<std::shared_mutex> lk(g_seg_mu);
    {
      for (uint64_t si = 0; si < S; si++) {
        auto it = g_segs.find(seg_keys[si]);
        if (it == g_segs.end()) return fail(PG_E_NOTFOUND, "segment %llu not resident", (unsigned long long)seg_keys[si]);
        auto c = it->second->cols.find(col_id);
        if (c == it->second->cols.end() || !c->second.has_dict)
          return fail(PG_E_NOTFOUND, "segment %llu has no dictionary for column %u", (unsigned long long)seg_keys[si], col_id);
        if (c->second.dtype != data_type)
          return fail(PG_E_INVALID, "column %u's dictionary holds type %u, the literals %u", col_id, c->second.dtype, data_type);
        jobs[si].dict = c->second.dict.p;
        jobs[si].card = c->second.card;
      }
    }
    const uint64_t vb = n * (data_type == PG_INT || data_type == PG_FLOAT ? 4 : 8);
    hipStream_t s = thread_stream();
    Scratch sc(s);
    DictLookupJob* dj = sc.get<DictLookupJob>(S, rc);
    uint8_t* dv = sc.get<uint8_t>(vb, rc);
    int32_t* dout = sc.get<int32_t>(S * n, rc);
    if (rc) return rc;
    HIP_CHECK(hipMemcpyAsync(dj, jobs.data(), S * sizeof(DictLookupJob), hipMemcpyHostToDevice, s));
    HIP_CHECK(hipMemcpyAsync(dv, values, vb, hipMemcpyHostToDevice, s));
    HIP_CHECK(launch_dict_lookup(dj, (uint32_t)S, dv, (uint32_t)n, data_type, dout, s));
    HIP_CHECK(hipMemcpyAsync(out_ids, dout, S * n * 4, hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
    // compact each segment's row in place: the found ids, ascending (the literals and the dictionary are sorted)
    for (uint64_t si = 0; si < S; si++) {
      int32_t* row = out_ids + si * n;
      uint32_t k = 0;
      for (uint64_t i = 0; i < n; i++)
        if (row[i] >= 0) row[k++] = row[i];
      out_counts[si] = k;
    }
    return PG_OK;
  } catch (const std::exception& e) {
    return fail(PG_E_NOMEM, "dictionary lookup failed: %s", e.what());
  }
}

int pg_execute(const pg_plan* plan, pg_result** out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  if (multi_device() && !t_is_worker) {  // the segments' logical devices, their states merged in the library
    pg_partials* p = nullptr;
    int rc = execute_partial_multi(plan, &p);
    if (rc) return rc;
    const pg_timing te = t_timing;
    const pg_trace tr = t_trace;
    rc = pg_partials_finalize(p, plan, out);
    pg_timing tf = t_timing;
    t_timing = te;
    t_timing.finalize_ms = tf.finalize_ms;
    t_timing.finalize_wall_ms = tf.finalize_wall_ms;
    t_trace = tr;
    pg_partials_free(p);
    return rc;
  }
  t_prof.n = 0;
  const double t_prof_start = wall_ms();
  pg_partials* p = nullptr;
  t_prefetch_state = true;  // the state is finalised right after: copy a small one back with the scan's counts
  int rc = pg_execute_partial(plan, &p);
  t_prefetch_state = false;
  if (rc) return rc;
  PG_PROF("execute");
  rc = pg_partials_finalize(p, plan, out);
  pg_partials_free(p);
  PG_PROF("finalize");
  host_prof_dump(t_prof.n ? t_prof_start : 0);
  return rc;
}

int pg_execute_image(const void* image, uint64_t n, pg_result** out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  try {
    PlanImage pi;
    const int rc = decode_image(image, n, pi);
    return rc ? rc : pg_execute(&pi.plan, out);
  } catch (const std::exception& e) {
    return fail(PG_E_NOMEM, "execute failed: %s", e.what());
  }
}

int pg_execute_partial_image(const void* image, uint64_t n, pg_partials** out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  try {
    PlanImage pi;
    const int rc = decode_image(image, n, pi);
    return rc ? rc : pg_execute_partial(&pi.plan, out);
  } catch (const std::exception& e) {
    return fail(PG_E_NOMEM, "execute failed: %s", e.what());
  }
}

int pg_partials_finalize_image(pg_partials* p, const void* image, uint64_t n, pg_result** out) {
  try {
    PlanImage pi;
    const int rc = decode_image(image, n, pi);
    return rc ? rc : pg_partials_finalize(p, &pi.plan, out);
  } catch (const std::exception& e) {
    return fail(PG_E_NOMEM, "finalize failed: %s", e.what());
  }
}

int pg_result_free(pg_result* r) {
  if (!r) return PG_OK;
  res_free(r->keys);
  res_free(r->values);
  res_free(r->counts);
  res_free(r->distinct_offsets);
  res_free(r->distinct_ids);
  free(r);
  return PG_OK;
}

int pg_chunk_decompress(uint32_t codec, const void* src, uint64_t src_len, void* dst, uint64_t dst_cap,
                        uint64_t* out_len) {
  if ((!src && src_len) || (!dst && dst_cap) || !out_len) return fail(PG_E_INVALID, "null argument");
  const char* why = "";
  const int rc = decompress_chunk(codec, (const uint8_t*)src, src_len, (uint8_t*)dst, dst_cap, out_len, &why);
  return rc ? fail(rc, "%s", why) : PG_OK;
}

int pg_last_trace(pg_trace* out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  *out = t_trace;
  return PG_OK;
}

int pg_last_timing(pg_timing* out) {
  if (!out) return fail(PG_E_INVALID, "null out");
  *out = t_timing;
  return PG_OK;
}

}  // extern "C"
