// pg_codec.hip -- host-side chunk decoders of raw (no-dictionary) forward indexes (libpinot_gpu).
//
// The reference stores a raw column in chunks compressed per ChunkCompressionType (SNAPPY / ZSTANDARD / LZ4 /
// LZ4_LENGTH_PREFIXED, pinot-segment-spi/.../compression/ChunkCompressionType.java:21-22; writer
// BaseChunkSVForwardIndexWriter, readers BaseChunkForwardIndexReader.java:56-102) and decompresses a chunk through
// ChunkDecompressor every time a reader touches it (io/compression/*Decompressor.java).  Here a chunk is decompressed
// once, when pg_column_upload makes the column resident (upload-time format conversion, like the byte swaps of the
// bit-packed indexes); the query path then reads plain typed values from HBM.
//
// The codecs are third-party libraries of the reference (snappy-java 1.1.8.2, lz4-java 1.8.0, zstd-jni 1.4.9-5,
// pom.xml:150-152) and are restated here from their published formats: the Snappy block format, the LZ4 block format,
// and Zstandard frames (RFC 8878: FSE / Huffman entropy stages, sequence execution with repeat offsets).  No
// dictionary-compressed zstd frames (Pinot never writes them).  Host code only: no kernels in this file.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/pinot_codec.h"

namespace pg {
namespace codec {

#define BAD(msg)    \
  do {              \
    *why = (msg);   \
    return PG_E_INVALID; \
  } while (0)

// ------------------------------------------------------------------------------------------ Snappy (block format)
static int snappy(const uint8_t* p, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out, const char** why) {
  uint64_t pos = 0, len = 0;
  for (int shift = 0;; shift += 7) {
    if (pos >= n || shift > 35) BAD("snappy: bad length header");
    const uint8_t b = p[pos++];
    len |= (uint64_t)(b & 0x7F) << shift;
    if (b < 0x80) break;
  }
  if (len > cap) BAD("snappy: chunk larger than its buffer");
  uint64_t op = 0;
  while (pos < n) {
    const uint8_t tag = p[pos++];
    uint64_t ln, off = 0;
    if ((tag & 3) == 0) {  // literal
      ln = tag >> 2;
      if (ln >= 60) {
        const uint32_t nb = (uint32_t)ln - 59;
        if (pos + nb > n) BAD("snappy: truncated literal length");
        ln = 0;
        for (uint32_t k = 0; k < nb; k++) ln |= (uint64_t)p[pos + k] << (8 * k);
        pos += nb;
      }
      ln += 1;
      if (pos + ln > n || op + ln > len) BAD("snappy: truncated literal");
      memcpy(dst + op, p + pos, ln);
      pos += ln;
      op += ln;
      continue;
    }
    if ((tag & 3) == 1) {  // copy, 1-byte offset
      if (pos + 1 > n) BAD("snappy: truncated copy");
      ln = ((tag >> 2) & 7) + 4;
      off = ((uint64_t)(tag >> 5) << 8) | p[pos];
      pos += 1;
    } else {  // copy, 2- or 4-byte offset
      const uint32_t nb = (tag & 3) == 2 ? 2 : 4;
      if (pos + nb > n) BAD("snappy: truncated copy");
      ln = (tag >> 2) + 1;
      for (uint32_t k = 0; k < nb; k++) off |= (uint64_t)p[pos + k] << (8 * k);
      pos += nb;
    }
    if (off == 0 || off > op || op + ln > len) BAD("snappy: copy out of range");
    for (uint64_t k = 0; k < ln; k++) dst[op + k] = dst[op + k - off];  // may overlap its own output
    op += ln;
  }
  if (op != len) BAD("snappy: decoded length differs from the header");
  *out = op;
  return PG_OK;
}

// ------------------------------------------------------------------------------------------ LZ4 (block format)
static int lz4_block(const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out, const char** why) {
  uint64_t ip = 0, op = 0;
  if (n == 0) BAD("lz4: empty block");
  for (;;) {
    if (ip >= n) BAD("lz4: block ends inside a sequence");
    const uint8_t token = src[ip++];
    uint64_t lit = token >> 4;
    if (lit == 15) {
      uint8_t b;
      do {
        if (ip >= n) BAD("lz4: truncated literal length");
        b = src[ip++];
        lit += b;
      } while (b == 255);
    }
    if (ip + lit > n || op + lit > cap) BAD("lz4: literals out of range");
    memcpy(dst + op, src + ip, lit);
    ip += lit;
    op += lit;
    if (ip == n) break;  // the last sequence carries literals only
    if (ip + 2 > n) BAD("lz4: truncated match offset");
    const uint64_t off = (uint64_t)src[ip] | ((uint64_t)src[ip + 1] << 8);
    ip += 2;
    if (off == 0 || off > op) BAD("lz4: match offset out of range");
    uint64_t ml = token & 15;
    if (ml == 15) {
      uint8_t b;
      do {
        if (ip >= n) BAD("lz4: truncated match length");
        b = src[ip++];
        ml += b;
      } while (b == 255);
    }
    ml += 4;
    if (op + ml > cap) BAD("lz4: match past the chunk");
    for (uint64_t k = 0; k < ml; k++) dst[op + k] = dst[op + k - off];
    op += ml;
  }
  *out = op;
  return PG_OK;
}

// ------------------------------------------------------------------------------------------ Zstandard (RFC 8878)

// Forward bit reader (FSE table descriptions): little-endian bit order, bit i = (p[i / 8] >> (i % 8)) & 1.
struct FwdBits {
  const uint8_t* p;
  uint64_t n, pos = 0;  // pos in bits
  uint32_t peek(uint32_t k) const {
    uint64_t v = 0;
    const uint64_t b = pos >> 3;
    for (uint32_t i = 0; i < 8 && b + i < n; i++) v |= (uint64_t)p[b + i] << (8 * i);
    return (uint32_t)((v >> (pos & 7)) & ((1ull << k) - 1));
  }
};

// Backward bit reader (Huffman / FSE streams): the stream ends with a 1-bit marker in its last byte; bits are read
// from the marker downwards, a read of k bits returning bits [bitpos - k, bitpos) as a number.  Bits below the start
// read as zeros and leave bitpos negative (the "overflow" the decoders test for).
struct BackBits {
  const uint8_t* p = nullptr;
  uint64_t n = 0;
  int64_t bitpos = 0;
  bool init(const uint8_t* q, uint64_t len) {
    p = q;
    n = len;
    if (!len || !q[len - 1]) return false;
    bitpos = (int64_t)(len - 1) * 8 + (31 - __builtin_clz((uint32_t)q[len - 1]));
    return true;
  }
  uint64_t get(int64_t start, uint32_t k) const {  // bits [start, start + k), start >= 0, k <= 57
    uint64_t v = 0;
    const uint64_t b = (uint64_t)start >> 3;
    for (uint32_t i = 0; i < 8 && b + i < n; i++) v |= (uint64_t)p[b + i] << (8 * i);
    return (v >> (start & 7)) & (k >= 64 ? ~0ull : ((1ull << k) - 1));
  }
  uint64_t peek(uint32_t k) const {
    if (!k) return 0;
    const int64_t s = bitpos - (int64_t)k;
    if (s >= 0) return get(s, k);
    if (bitpos <= 0) return 0;
    return get(0, (uint32_t)bitpos) << (uint32_t)(-s);
  }
  uint64_t read(uint32_t k) {
    const uint64_t v = peek(k);
    bitpos -= k;
    return v;
  }
  bool overflow() const { return bitpos < 0; }
};

struct FseEntry {
  uint16_t symbol;
  uint8_t nbits;
  uint16_t baseline;
};
struct FseTable {
  uint32_t log = 0;
  std::vector<FseEntry> t;
};

static int highbit(uint32_t x) { return 31 - __builtin_clz(x); }

// FSE decoding table from normalized counts (RFC 8878 4.1.1): "less than 1" symbols at the top, the others spread
// by the step (tableSize >> 1) + (tableSize >> 3) + 3, then per-state bit counts and baselines.
static int fse_build(const int16_t* norm, uint32_t nsym, uint32_t log, FseTable& T, const char** why) {
  const uint32_t size = 1u << log;
  T.log = log;
  T.t.assign(size, FseEntry{0, 0, 0});
  std::vector<uint32_t> next(nsym);
  uint32_t high = size - 1;
  for (uint32_t s = 0; s < nsym; s++) {
    if (norm[s] == -1) {
      T.t[high--].symbol = (uint16_t)s;
      next[s] = 1;
    } else {
      next[s] = (uint32_t)std::max<int>(norm[s], 0);
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
  uint32_t pos = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    for (int i = 0; i < norm[s]; i++) {
      T.t[pos].symbol = (uint16_t)s;
      do pos = (pos + step) & mask;
      while (pos > high);
    }
  }
  if (pos != 0) BAD("zstd: FSE distribution does not fill its table");
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t s = T.t[u].symbol;
    const uint32_t ns = next[s]++;
    const uint32_t nb = log - (uint32_t)highbit(ns);
    T.t[u].nbits = (uint8_t)nb;
    T.t[u].baseline = (uint16_t)((ns << nb) - size);
  }
  return PG_OK;
}

// FSE table description (RFC 8878 4.1.1): accuracy log, then normalized counts with zero-repeat flags.  Returns the
// bytes consumed in *used.
static int fse_read_table(const uint8_t* p, uint64_t n, uint32_t max_sym, uint32_t max_log, FseTable& T,
                          uint64_t* used, const char** why) {
  FwdBits br{p, n};
  if (n < 1) BAD("zstd: empty FSE table description");
  const uint32_t log = br.peek(4) + 5;
  br.pos += 4;
  if (log > max_log) BAD("zstd: FSE accuracy log too large");
  int16_t norm[256] = {0};
  int32_t remaining = (1 << log) + 1, threshold = 1 << log;
  uint32_t nbits = log + 1, sym = 0;
  bool prev0 = false;
  while (remaining > 1 && sym <= max_sym) {
    if (prev0) {  // repeat flags of zero probabilities
      for (;;) {
        const uint32_t f = br.peek(2);
        br.pos += 2;
        sym += f;
        if (f != 3) break;
      }
      if (sym > max_sym) break;
    }
    const int32_t mx = (2 * threshold - 1) - remaining;
    const uint32_t v = br.peek(nbits);
    int32_t count;
    if ((int32_t)(v & (threshold - 1)) < mx) {
      count = (int32_t)(v & (threshold - 1));
      br.pos += nbits - 1;
    } else {
      count = (int32_t)(v & (2 * threshold - 1));
      if (count >= threshold) count -= mx;
      br.pos += nbits;
    }
    count--;  // -1: "less than 1"
    remaining -= count < 0 ? -count : count;
    norm[sym++] = (int16_t)count;
    prev0 = count == 0;
    while (remaining < threshold) {
      nbits--;
      threshold >>= 1;
    }
    if ((br.pos >> 3) > n) BAD("zstd: truncated FSE table description");
  }
  if (remaining != 1 || sym > max_sym + 1) BAD("zstd: bad FSE normalized counts");
  *used = (br.pos + 7) >> 3;
  return fse_build(norm, std::max<uint32_t>(sym, 1), log, T, why);
}

struct HufTable {
  uint32_t max_bits = 0;
  std::vector<uint16_t> sym;  // [1 << max_bits]
  std::vector<uint8_t> nb;
};

// Huffman tree description (RFC 8878 4.2.1): weights (FSE-compressed or 4-bit direct), the last one implied, then
// the decoding table of prefix codes assigned by rank (weight ascending, symbols ascending within a weight).
static int huf_read_table(const uint8_t* p, uint64_t n, HufTable& H, uint64_t* used, const char** why) {
  if (n < 1) BAD("zstd: empty Huffman tree description");
  uint8_t w[256] = {0};
  uint32_t nw = 0;
  const uint32_t hb = p[0];
  if (hb < 128) {  // FSE-compressed weights, two interleaved states
    if (1 + (uint64_t)hb > n) BAD("zstd: truncated Huffman weights");
    FseTable T;
    uint64_t tu = 0;
    int rc = fse_read_table(p + 1, hb, 255, 6, T, &tu, why);
    if (rc) return rc;
    if (tu >= hb) BAD("zstd: Huffman weight stream missing");
    BackBits bb;
    if (!bb.init(p + 1 + tu, hb - tu)) BAD("zstd: bad Huffman weight stream");
    uint32_t s1 = (uint32_t)bb.read(T.log), s2 = (uint32_t)bb.read(T.log);
    for (;;) {
      if (nw >= 255) BAD("zstd: too many Huffman weights");
      w[nw++] = (uint8_t)T.t[s1].symbol;
      s1 = T.t[s1].baseline + (uint32_t)bb.read(T.t[s1].nbits);
      if (bb.overflow()) {
        w[nw++] = (uint8_t)T.t[s2].symbol;
        break;
      }
      if (nw >= 255) BAD("zstd: too many Huffman weights");
      w[nw++] = (uint8_t)T.t[s2].symbol;
      s2 = T.t[s2].baseline + (uint32_t)bb.read(T.t[s2].nbits);
      if (bb.overflow()) {
        w[nw++] = (uint8_t)T.t[s1].symbol;
        break;
      }
    }
    *used = 1 + hb;
  } else {  // direct: 4 bits per weight
    nw = hb - 127;
    const uint64_t nb = (nw + 1) / 2;
    if (1 + nb > n) BAD("zstd: truncated Huffman weights");
    for (uint32_t i = 0; i < nw; i++) w[i] = (i & 1) ? (p[1 + i / 2] & 15) : (p[1 + i / 2] >> 4);
    *used = 1 + nb;
  }
  uint32_t sum = 0;
  for (uint32_t i = 0; i < nw; i++) {
    if (w[i] > 12) BAD("zstd: Huffman weight out of range");
    if (w[i]) sum += 1u << (w[i] - 1);
  }
  if (!sum) BAD("zstd: empty Huffman tree");
  if (nw > 255) BAD("zstd: too many Huffman weights");  // the implied last weight is the 256th symbol at most
  const uint32_t max_bits = (uint32_t)highbit(sum) + 1;
  const uint32_t left = (1u << max_bits) - sum;
  if (left & (left - 1)) BAD("zstd: Huffman weights do not complete a tree");
  w[nw++] = (uint8_t)(highbit(left) + 1);  // the implied last weight
  if (max_bits > 12) BAD("zstd: Huffman table too deep");
  uint32_t rank[13] = {0};
  for (uint32_t i = 0; i < nw; i++) rank[w[i]]++;
  uint32_t start[13] = {0}, acc = 0;
  for (uint32_t k = 1; k <= max_bits; k++) {
    start[k] = acc;
    acc += rank[k] << (k - 1);
  }
  H.max_bits = max_bits;
  H.sym.assign(1u << max_bits, 0);
  H.nb.assign(1u << max_bits, 0);
  for (uint32_t s = 0; s < nw; s++) {
    if (!w[s]) continue;
    const uint32_t len = 1u << (w[s] - 1);
    for (uint32_t u = start[w[s]]; u < start[w[s]] + len; u++) {
      H.sym[u] = (uint16_t)s;
      H.nb[u] = (uint8_t)(max_bits + 1 - w[s]);
    }
    start[w[s]] += len;
  }
  return PG_OK;
}

static int huf_stream(const HufTable& H, const uint8_t* p, uint64_t n, uint8_t* out, uint64_t cnt, const char** why) {
  BackBits bb;
  if (!bb.init(p, n)) BAD("zstd: bad Huffman stream");
  for (uint64_t i = 0; i < cnt; i++) {
    const uint32_t v = (uint32_t)bb.peek(H.max_bits);
    out[i] = (uint8_t)H.sym[v];
    bb.bitpos -= H.nb[v];
  }
  if (bb.bitpos != 0) BAD("zstd: Huffman stream not fully consumed");
  return PG_OK;
}

// Predefined sequence code distributions and the literal / match length code tables (RFC 8878 3.1.1.3.2).
static const int16_t kLLDefault[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                       2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t kMLDefault[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t kOFDefault[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,    15,    16,    18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
static const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,  16,   17,   18,   19,   20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,  34,   35,   37,   39,   41,
                                     43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
static const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

struct ZState {  // per frame: tables carried across blocks (Treeless literals, Repeat_Mode sequences), repeat offsets
  HufTable huf;
  bool has_huf = false;
  FseTable ll, of, ml;
  bool has_ll = false, has_of = false, has_ml = false;
  uint64_t rep[3] = {1, 4, 8};
};

static int seq_table(uint32_t mode, const uint8_t* p, uint64_t n, uint64_t* pos, const int16_t* dflt, uint32_t dsym,
                     uint32_t dlog, uint32_t max_sym, uint32_t max_log, FseTable& T, bool& has, const char** why) {
  switch (mode) {
    case 0: {  // Predefined_Mode
      int rc = fse_build(dflt, dsym, dlog, T, why);
      if (rc) return rc;
      break;
    }
    case 1: {  // RLE_Mode: one symbol, accuracy log 0
      if (*pos >= n) BAD("zstd: truncated RLE sequence code");
      const uint32_t s = p[(*pos)++];
      if (s > max_sym) BAD("zstd: RLE sequence code out of range");
      T.log = 0;
      T.t.assign(1, FseEntry{(uint16_t)s, 0, 0});
      break;
    }
    case 2: {  // FSE_Compressed_Mode
      uint64_t used = 0;
      int rc = fse_read_table(p + *pos, n - *pos, max_sym, max_log, T, &used, why);
      if (rc) return rc;
      *pos += used;
      break;
    }
    default:  // Repeat_Mode
      if (!has) BAD("zstd: repeat mode without a previous table");
      break;
  }
  has = true;
  return PG_OK;
}

static int zstd_block(ZState& Z, const uint8_t* p, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* op,
                      std::vector<uint8_t>& lit, const char** why) {
  // ---- literals section
  if (n < 1) BAD("zstd: empty compressed block");
  const uint32_t ltype = p[0] & 3, sf = (p[0] >> 2) & 3;
  uint64_t pos = 0, regen = 0, csize = 0;
  uint32_t streams = 1;
  if (ltype <= 1) {  // Raw / RLE
    if (sf == 0 || sf == 2) { regen = p[0] >> 3; pos = 1; }
    else if (sf == 1) { if (n < 2) BAD("zstd: truncated literals header"); regen = (p[0] >> 4) + ((uint64_t)p[1] << 4); pos = 2; }
    else { if (n < 3) BAD("zstd: truncated literals header"); regen = (p[0] >> 4) + ((uint64_t)p[1] << 4) + ((uint64_t)p[2] << 12); pos = 3; }
    lit.resize(regen);
    if (ltype == 0) {
      if (pos + regen > n) BAD("zstd: truncated raw literals");
      if (regen) memcpy(lit.data(), p + pos, regen);
      pos += regen;
    } else {
      if (pos + 1 > n) BAD("zstd: truncated RLE literals");
      memset(lit.data(), p[pos], regen);
      pos += 1;
    }
  } else {  // Compressed / Treeless
    uint32_t hsize, bits;
    if (sf <= 1) { hsize = 3; bits = 10; streams = sf == 0 ? 1 : 4; }
    else if (sf == 2) { hsize = 4; bits = 14; streams = 4; }
    else { hsize = 5; bits = 18; streams = 4; }
    if (n < hsize) BAD("zstd: truncated literals header");
    uint64_t h = 0;
    for (uint32_t i = 0; i < hsize; i++) h |= (uint64_t)p[i] << (8 * i);
    regen = (h >> 4) & ((1ull << bits) - 1);
    csize = (h >> (4 + bits)) & ((1ull << bits) - 1);
    pos = hsize;
    if (pos + csize > n) BAD("zstd: truncated compressed literals");
    const uint8_t* q = p + pos;
    uint64_t qn = csize;
    if (ltype == 2) {
      uint64_t used = 0;
      int rc = huf_read_table(q, qn, Z.huf, &used, why);
      if (rc) return rc;
      Z.has_huf = true;
      q += used;
      qn -= used;
    } else if (!Z.has_huf) {
      BAD("zstd: treeless literals without a previous Huffman table");
    }
    lit.resize(regen);
    if (streams == 1) {
      int rc = huf_stream(Z.huf, q, qn, lit.data(), regen, why);
      if (rc) return rc;
    } else {
      if (qn < 6) BAD("zstd: truncated literal jump table");
      const uint64_t s1 = q[0] | ((uint64_t)q[1] << 8), s2 = q[2] | ((uint64_t)q[3] << 8), s3 = q[4] | ((uint64_t)q[5] << 8);
      if (6 + s1 + s2 + s3 > qn) BAD("zstd: literal streams past their section");
      const uint64_t s4 = qn - 6 - s1 - s2 - s3, per = (regen + 3) / 4;
      if (regen < 3 * per) BAD("zstd: literal stream sizes inconsistent");
      const uint8_t* st = q + 6;
      const uint64_t sz[4] = {s1, s2, s3, s4}, cnt[4] = {per, per, per, regen - 3 * per};
      uint64_t o = 0;
      for (int k = 0; k < 4; k++) {
        int rc = huf_stream(Z.huf, st, sz[k], lit.data() + o, cnt[k], why);
        if (rc) return rc;
        st += sz[k];
        o += cnt[k];
      }
    }
    pos += csize;
  }
  // ---- sequences section
  if (pos >= n) BAD("zstd: missing sequences section");
  uint64_t nseq = p[pos++];
  if (nseq >= 128) {
    if (nseq < 255) {
      if (pos >= n) BAD("zstd: truncated sequence count");
      nseq = ((nseq - 128) << 8) + p[pos++];
    } else {
      if (pos + 2 > n) BAD("zstd: truncated sequence count");
      nseq = p[pos] + ((uint64_t)p[pos + 1] << 8) + 0x7F00;
      pos += 2;
    }
  }
  uint64_t li = 0;  // literals consumed
  if (nseq) {
    if (pos >= n) BAD("zstd: missing symbol compression modes");
    const uint8_t modes = p[pos++];
    if (modes & 3) BAD("zstd: reserved bits in the compression modes");
    int rc = seq_table(modes >> 6, p, n, &pos, kLLDefault, 36, 6, 35, 9, Z.ll, Z.has_ll, why);
    if (!rc) rc = seq_table((modes >> 4) & 3, p, n, &pos, kOFDefault, 29, 5, 31, 8, Z.of, Z.has_of, why);
    if (!rc) rc = seq_table((modes >> 2) & 3, p, n, &pos, kMLDefault, 53, 6, 52, 9, Z.ml, Z.has_ml, why);
    if (rc) return rc;
    BackBits bb;
    if (pos >= n || !bb.init(p + pos, n - pos)) BAD("zstd: bad sequence bitstream");
    uint32_t sll = (uint32_t)bb.read(Z.ll.log), sof = (uint32_t)bb.read(Z.of.log), sml = (uint32_t)bb.read(Z.ml.log);
    for (uint64_t i = 0; i < nseq; i++) {
      const uint32_t llc = Z.ll.t[sll].symbol, ofc = Z.of.t[sof].symbol, mlc = Z.ml.t[sml].symbol;
      if (llc > 35 || mlc > 52 || ofc > 31) BAD("zstd: sequence code out of range");
      const uint64_t ofv = (1ull << ofc) + bb.read(ofc);
      const uint64_t ml = kMLBase[mlc] + bb.read(kMLBits[mlc]);
      const uint64_t ll = kLLBase[llc] + bb.read(kLLBits[llc]);
      uint64_t off;
      if (ofv > 3) {
        off = ofv - 3;
        Z.rep[2] = Z.rep[1];
        Z.rep[1] = Z.rep[0];
        Z.rep[0] = off;
      } else {  // repeat offsets; a zero literal length shifts the codes by one (RFC 8878 3.1.1.5)
        const uint32_t code = (uint32_t)ofv - 1 + (ll == 0 ? 1 : 0);
        if (code == 0) {
          off = Z.rep[0];
        } else {
          off = code == 3 ? Z.rep[0] - 1 : Z.rep[code];
          if (code != 1) Z.rep[2] = Z.rep[1];
          Z.rep[1] = Z.rep[0];
          Z.rep[0] = off;
        }
      }
      if (li + ll > lit.size() || *op + ll + ml > cap) BAD("zstd: sequence past its buffers");
      memcpy(dst + *op, lit.data() + li, ll);
      li += ll;
      *op += ll;
      if (off == 0 || off > *op) BAD("zstd: match offset out of range");
      for (uint64_t k = 0; k < ml; k++) dst[*op + k] = dst[*op + k - off];
      *op += ml;
      if (i + 1 < nseq) {  // state updates: literal lengths, match lengths, offsets
        sll = Z.ll.t[sll].baseline + (uint32_t)bb.read(Z.ll.t[sll].nbits);
        sml = Z.ml.t[sml].baseline + (uint32_t)bb.read(Z.ml.t[sml].nbits);
        sof = Z.of.t[sof].baseline + (uint32_t)bb.read(Z.of.t[sof].nbits);
      }
    }
    if (bb.bitpos != 0) BAD("zstd: sequence bitstream not fully consumed");
  }
  const uint64_t rest = lit.size() - li;  // the literals after the last sequence
  if (*op + rest > cap) BAD("zstd: literals past the chunk");
  if (rest) memcpy(dst + *op, lit.data() + li, rest);
  *op += rest;
  return PG_OK;
}

static int zstd(const uint8_t* p, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out, const char** why) {
  uint64_t pos = 0, op = 0;
  std::vector<uint8_t> lit;
  while (pos < n) {
    if (pos + 4 > n) BAD("zstd: truncated frame magic");
    const uint32_t magic = p[pos] | (p[pos + 1] << 8) | (p[pos + 2] << 16) | ((uint32_t)p[pos + 3] << 24);
    pos += 4;
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (pos + 4 > n) BAD("zstd: truncated skippable frame");
      const uint64_t sz = p[pos] | (p[pos + 1] << 8) | (p[pos + 2] << 16) | ((uint64_t)p[pos + 3] << 24);
      pos += 4 + sz;
      continue;
    }
    if (magic != 0xFD2FB528u) BAD("zstd: bad frame magic");
    if (pos >= n) BAD("zstd: truncated frame header");
    const uint8_t fhd = p[pos++];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
    if (fhd & 8) BAD("zstd: reserved frame header bit");
    static const uint32_t did_size[4] = {0, 1, 2, 4};
    static const uint32_t fcs_size[4] = {0, 2, 4, 8};
    const uint32_t fs = fcs_flag == 0 ? (single ? 1 : 0) : fcs_size[fcs_flag];
    // window descriptor + dictionary id + frame content size, all inside the chunk before any of them is read
    if ((uint64_t)pos + (single ? 0 : 1) + did_size[did_flag] + fs > n) BAD("zstd: truncated frame header");
    if (!single) pos += 1;  // window descriptor (the whole chunk is decoded into one buffer)
    uint64_t did = 0;
    for (uint32_t i = 0; i < did_size[did_flag]; i++) did |= (uint64_t)p[pos + i] << (8 * i);
    pos += did_size[did_flag];
    if (did) return PG_E_UNSUPPORTED;  // dictionaries: never written by Pinot
    pos += fs;
    ZState Z;
    for (;;) {
      if (pos + 3 > n) BAD("zstd: truncated block header");
      const uint32_t bh = p[pos] | (p[pos + 1] << 8) | ((uint32_t)p[pos + 2] << 16);
      pos += 3;
      const uint32_t last = bh & 1, btype = (bh >> 1) & 3, bsize = bh >> 3;
      if (btype == 0) {  // Raw_Block
        if (pos + bsize > n || op + bsize > cap) BAD("zstd: raw block out of range");
        memcpy(dst + op, p + pos, bsize);
        op += bsize;
        pos += bsize;
      } else if (btype == 1) {  // RLE_Block: one byte, Block_Size times
        if (pos + 1 > n || op + bsize > cap) BAD("zstd: RLE block out of range");
        memset(dst + op, p[pos], bsize);
        op += bsize;
        pos += 1;
      } else if (btype == 2) {
        if (pos + bsize > n) BAD("zstd: truncated compressed block");
        int rc = zstd_block(Z, p + pos, bsize, dst, cap, &op, lit, why);
        if (rc) return rc;
        pos += bsize;
      } else {
        BAD("zstd: reserved block type");
      }
      if (last) break;
    }
    if (checksum) pos += 4;  // XXH64 of the content (not verified)
  }
  *out = op;
  return PG_OK;
}

}  // namespace codec

// One chunk of a raw forward index (ChunkDecompressor.decompress); *why receives the reason of a failure.
int decompress_chunk(uint32_t kind, const uint8_t* src, uint64_t n, uint8_t* dst, uint64_t cap, uint64_t* out,
                     const char** why) {
  *why = "";
  switch (kind) {
    case PG_CODEC_PASS_THROUGH:
      if (n > cap) {
        *why = "pass-through chunk larger than its buffer";
        return PG_E_INVALID;
      }
      memcpy(dst, src, n);
      *out = n;
      return PG_OK;
    case PG_CODEC_SNAPPY: return codec::snappy(src, n, dst, cap, out, why);
    case PG_CODEC_ZSTANDARD: {
      const int rc = codec::zstd(src, n, dst, cap, out, why);
      if (rc == PG_E_UNSUPPORTED) *why = "zstd: dictionary-compressed frame";
      return rc;
    }
    case PG_CODEC_LZ4: return codec::lz4_block(src, n, dst, cap, out, why);
    case PG_CODEC_LZ4_LENGTH_PREFIXED: {  // LZ4CompressorWithLength: 4-byte little-endian original length + block
      if (n < 4) {
        *why = "lz4: missing length prefix";
        return PG_E_INVALID;
      }
      const uint64_t len = src[0] | (src[1] << 8) | (src[2] << 16) | ((uint64_t)src[3] << 24);
      if (len > cap) {
        *why = "lz4: chunk larger than its buffer";
        return PG_E_INVALID;
      }
      const int rc = codec::lz4_block(src + 4, n - 4, dst, len, out, why);
      if (!rc && *out != len) {
        *why = "lz4: decoded length differs from the prefix";
        return PG_E_INVALID;
      }
      return rc;
    }
    default:
      *why = "unknown chunk compression type";
      return PG_E_UNSUPPORTED;
  }
}

}  // namespace pg
