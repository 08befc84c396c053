// pg_wide.hip -- group keys wider than a packed 62-bit key (gfx950): the device form of the reference's
// ArrayMapBasedHolder.
//
// DictionaryBasedGroupKeyGenerator switches to ArrayMapBasedHolder when the product of the key cardinalities overflows
// a long (query/aggregation/groupby/DictionaryBasedGroupKeyGenerator.java:117-147, holder :777-860): the raw key is
// the int[] of the doc's dictIds and an Object2IntOpenHashMap<IntArray> gives it a group id.  Here the same role is
// split in two so that the fused scan keeps its one-word keys:
//   1. intern_kernel: for every doc of every segment, the K table-global key ids (value offsets / keymaps, exactly as
//      the scan forms them) are hashed and interned into an open-addressing table of tuples; the doc's tuple slot is
//      written to a per-segment uint32 column.  Slots are claimed with a 64-bit CAS on a tag word (0 = free, 1 = being
//      written, else the tuple's hash | 2); the claimer writes the tuple, releases, then publishes the tag, and a lane
//      that reads tag 1 re-reads it in its next loop iteration (the writer finishes within its own iteration, so a
//      wave never waits on itself).  Tuples merge segments by VALUE, like packed keys do.
//   2. the fused scan groups by that column as one key whose id space is the table's slots; the runtime maps the
//      finished groups' slots back to their tuples (gather_tuples_kernel) for the result keys and the ORDER BY.
// numGroupsLimit and first-seen truncation then apply per (segment, tuple slot) exactly as for packed keys.
// Integer / atomic work bound by HBM latency; no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "pg_aux.h"

namespace pg {

namespace {

__device__ __forceinline__ uint32_t unpack_word(const uint32_t* w, uint32_t idx, uint32_t b) {
  // FixedBitIntReader.readUnchecked on the native-word image (the column keeps 4 zero words of tail padding)
  const uint64_t p = (uint64_t)idx * b;
  const uint64_t k = p >> 5;
  const uint64_t win = ((uint64_t)w[k] << 32) | (uint64_t)w[k + 1];
  return (uint32_t)(win >> (64u - ((uint32_t)p & 31u) - b)) & (0xFFFFFFFFu >> (32u - b));
}

// table-global key id of dictId `id` (the scan's key_of): ~0 when the id is outside the dictionary
__device__ __forceinline__ uint64_t wide_key_of(uint32_t kind, int64_t base, const ColDesc& c, uint32_t id) {
  if (id >= c.card) return ~0ull;
  if (kind == PG_KEY_KEYMAP) return (uint64_t)(uint32_t)c.keymap[id];
  int64_t v;
  if (c.decoded) v = c.vbase + (int64_t)id;
  else v = c.dtype == PG_INT ? (int64_t)((const int32_t*)c.dict)[id] : ((const int64_t*)c.dict)[id];
  return (uint64_t)(v - base);
}

// The tuple t[k * ts] (k < K, table-global ids, hash h) -> its slot in the table: claimed (tag 1), written, then
// published with its tag; a reader seeing the tag compares the stored tuple.  0xFFFFFFFF when the table is over its
// fill budget.
__device__ __forceinline__ uint32_t intern_probe(const WideSpec& w, const uint32_t* t, uint32_t ts, uint64_t h) {
  const uint32_t K = w.K;
  const unsigned long long tag = h | 2ull;
  uint64_t slot = (h >> 7) & w.mask;
  uint32_t res = 0xFFFFFFFFu;
  for (uint64_t n = 0; n <= w.mask;) {
    unsigned long long cur = __hip_atomic_load(&w.tags[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == 0ull) {
      if (__hip_atomic_load(w.fill, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= w.max_fill) break;
      const unsigned long long prev = atomicCAS(&w.tags[slot], 0ull, 1ull);
      if (prev == 0ull) {
        for (uint32_t k = 0; k < K; k++) w.tuples[slot * K + k] = t[k * ts];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_store(&w.tags[slot], tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicAdd(w.fill, 1u);
        res = (uint32_t)slot;
        break;
      }
      cur = prev;
    }
    if (cur == 1ull) continue;  // claimed, tuple not yet published: read the tag again
    if (cur == tag) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      bool eq = true;
      for (uint32_t k = 0; k < K; k++) eq &= w.tuples[slot * K + k] == t[k * ts];
      if (eq) {
        res = (uint32_t)slot;
        break;
      }
    }
    slot = (slot + 1) & w.mask;
    n++;
  }
  return res;
}

// the tuple hash of the intern table (row-major tuple t[k * ts])
__device__ __forceinline__ uint64_t tuple_hash(const uint32_t* t, uint32_t ts, uint32_t K) {
  uint64_t h = 0x9E3779B97F4A7C15ull;
  for (uint32_t k = 0; k < K; k++) h = mix64(h ^ ((uint64_t)t[k * ts] + 0x632BE59BD9B4E019ull * (k + 1)));
  return h;
}

constexpr int kWideBlock = 256;

__global__ __launch_bounds__(kWideBlock) void intern_kernel(WideSpec w) {
  extern __shared__ uint32_t row[];  // [K][kWideBlock]: this lane's tuple, column-major (no bank conflicts)
  const uint32_t seg = blockIdx.y, tid = threadIdx.x, K = w.K;
  const uint32_t nd = w.num_docs[seg];
  uint32_t* out = w.out[seg];
  const ColDesc* kc = w.keycols + (uint64_t)seg * K;
  for (uint64_t d0 = (uint64_t)blockIdx.x * kWideBlock; d0 < nd; d0 += (uint64_t)gridDim.x * kWideBlock) {
    const uint32_t d = (uint32_t)d0 + tid;
    if (d >= nd) continue;  // no barrier below: lanes past the segment just skip
    uint64_t h = 0x9E3779B97F4A7C15ull;
    bool ok = true;
    for (uint32_t k = 0; k < K; k++) {
      const ColDesc c = kc[k];
      const uint32_t id = c.bits ? unpack_word(c.words, d, c.bits) : d;  // bits 0: raw values indexed by doc
      const uint64_t kid = wide_key_of(w.key_kind[k], w.key_base[k], c, id);
      ok &= kid < w.key_card[k];
      row[k * kWideBlock + tid] = (uint32_t)kid;
      h = mix64(h ^ (kid + 0x632BE59BD9B4E019ull * (k + 1)));
    }
    if (!ok) {  // never expected: the host proved the key ranges; the scan then rejects the doc's slot too
      atomicOr(w.err, 1u);
      out[d] = 0xFFFFFFFFu;
      continue;
    }
    const uint32_t res = intern_probe(w, row + tid, kWideBlock, h);
    if (res == 0xFFFFFFFFu) atomicOr(w.err, 4u);  // over the fill budget: the runtime reruns with a larger table
    out[d] = res;
  }
}

__global__ void gather_tuples_kernel(const uint32_t* __restrict__ tuples, uint32_t K, const uint64_t* __restrict__ slots,
                                     uint64_t n, uint32_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * K) return;
  const uint64_t g = i / K, k = i - g * K;
  out[i] = tuples[slots[g] * K + k];
}

// Cross-state merge of wide keys (pg_partials_export / pg_partials_merge): a state's slots are local, so the rows
// travel with their tuples (table-global key ids, comparable on every GPU) and are re-interned on the owner.
// owner[i] = the part of exchange row i's tuple (its key word is the slot of the tuple: pg_key_owner's mix of the
// tuple hash)
__global__ void wide_owner_kernel(const uint32_t* __restrict__ tuples, uint32_t K, const uint8_t* __restrict__ rows,
                                  uint64_t rb, uint64_t n, uint32_t parts, uint32_t* __restrict__ owner) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t slot = *(const uint64_t*)(rows + i * rb);
  const uint64_t h = tuple_hash(tuples + slot * K, 1, K);
  owner[i] = (uint32_t)((mix64(h ^ 0x9E3779B97F4A7C15ull) >> 32) % parts);
}
// dst[i] = { rows[i] (rb bytes) | the tuple of its key's slot (K uint32, padded to 8 bytes) }, rbw bytes per row
__global__ void widen_rows_kernel(const uint8_t* __restrict__ rows, uint64_t rb, const uint32_t* __restrict__ tuples,
                                  uint32_t K, uint64_t n, uint8_t* __restrict__ dst, uint64_t rbw) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t* r = (const uint64_t*)(rows + i * rb);
  uint64_t* d = (uint64_t*)(dst + i * rbw);
  for (uint64_t k = 0; k < rb / 8; k++) d[k] = r[k];
  uint32_t* t = (uint32_t*)(dst + i * rbw + rb);
  for (uint32_t k = 0; k < K; k++) t[k] = tuples[r[0] * K + k];
  if (K & 1u) t[K] = 0u;
}
// out[i] = rows[i]'s state row (rb bytes) with its key replaced by the slot its tuple interns to in `w`
__global__ void intern_rows_kernel(WideSpec w, const uint8_t* __restrict__ rows, uint64_t n, uint64_t rb, uint64_t rbw,
                                   uint8_t* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* t = (const uint32_t*)(rows + i * rbw + rb);
  const uint32_t slot = intern_probe(w, t, 1, tuple_hash(t, 1, w.K));
  const uint64_t* r = (const uint64_t*)(rows + i * rbw);
  uint64_t* d = (uint64_t*)(out + i * rb);
  if (slot == 0xFFFFFFFFu) {
    atomicOr(w.err, 4u);
    d[0] = ~0ull;  // never merged: the call fails
  } else {
    d[0] = slot;
  }
  for (uint64_t k = 1; k < rb / 8; k++) d[k] = r[k];
}

}  // namespace

hipError_t launch_wide_owner(const uint32_t* tuples, uint32_t K, const uint8_t* rows, uint64_t rb, uint64_t n,
                             uint32_t parts, uint32_t* owner, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(wide_owner_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tuples, K, rows, rb, n, parts,
                     owner);
  return hipGetLastError();
}
hipError_t launch_widen_rows(const uint8_t* rows, uint64_t rb, const uint32_t* tuples, uint32_t K, uint64_t n,
                             uint8_t* dst, uint64_t rbw, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(widen_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, rows, rb, tuples, K, n, dst,
                     rbw);
  return hipGetLastError();
}
hipError_t launch_intern_rows(const WideSpec& w, const uint8_t* rows, uint64_t n, uint64_t rb, uint64_t rbw,
                              uint8_t* out, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(intern_rows_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, w, rows, n, rb, rbw, out);
  return hipGetLastError();
}

hipError_t launch_intern_tuples(const WideSpec& w, uint32_t max_docs, hipStream_t s) {
  if (!w.num_segments || !max_docs) return hipSuccess;
  const uint32_t bx = std::min<uint32_t>((max_docs + kWideBlock - 1) / kWideBlock, 2048u);
  hipLaunchKernelGGL(intern_kernel, dim3(bx, w.num_segments), dim3(kWideBlock), (size_t)w.K * kWideBlock * 4, s, w);
  return hipGetLastError();
}

hipError_t launch_gather_tuples(const uint32_t* tuples, uint32_t K, const uint64_t* slots, uint64_t n, uint32_t* out,
                                hipStream_t s) {
  if (!n || !K) return hipSuccess;
  const uint64_t total = n * K;
  hipLaunchKernelGGL(gather_tuples_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, tuples, K, slots, n,
                     out);
  return hipGetLastError();
}

}  // namespace pg
