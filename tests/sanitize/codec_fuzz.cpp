// Sanitizer harness (test infrastructure, CPU only): the chunk decoders of pg_codec.hip compiled as plain C++ with
// -fsanitize=address,undefined (tests/sanitize/Makefile) and fed valid chunks plus truncated, bit-flipped and
// overwritten variants of them.  Every input and output buffer is an exact-size heap block, so a read past the chunk or
// a write past the caller's capacity is an AddressSanitizer report (the harness then aborts: -fno-sanitize-recover).
//
// Corpus records (little-endian, written by tests/test_sanitizers.py): u32 codec | u64 n_orig | u64 n_comp | orig | comp.
// Usage: codec_fuzz <corpus> [mutations per record]
#include "../../pinot_amd/csrc/pg_codec.hip"

#include <cstdio>
#include <memory>
#include <random>

namespace {

struct Rec {
  uint32_t codec;
  std::vector<uint8_t> orig, comp;
};

bool read_corpus(const char* path, std::vector<Rec>& out) {
  FILE* f = fopen(path, "rb");
  if (!f) return false;
  for (;;) {
    Rec r;
    uint64_t no, nc;
    if (fread(&r.codec, 4, 1, f) != 1) break;
    if (fread(&no, 8, 1, f) != 1 || fread(&nc, 8, 1, f) != 1) { fclose(f); return false; }
    r.orig.resize(no);
    r.comp.resize(nc);
    if ((no && fread(r.orig.data(), 1, no, f) != no) || (nc && fread(r.comp.data(), 1, nc, f) != nc)) { fclose(f); return false; }
    out.push_back(std::move(r));
  }
  fclose(f);
  return true;
}

// decode `src` into an exact `cap`-byte heap block; returns the status
int decode(uint32_t codec, const std::vector<uint8_t>& src, uint64_t cap, std::vector<uint8_t>* got) {
  std::unique_ptr<uint8_t[]> in(new uint8_t[src.size() ? src.size() : 1]);
  if (!src.empty()) memcpy(in.get(), src.data(), src.size());
  std::unique_ptr<uint8_t[]> dst(new uint8_t[cap ? cap : 1]);
  uint64_t n = 0;
  const char* why = "";
  const int rc = pg::decompress_chunk(codec, src.empty() ? nullptr : in.get(), src.size(), dst.get(), cap, &n, &why);
  if (!rc && n > cap) { fprintf(stderr, "decoded %llu bytes into %llu\n", (unsigned long long)n, (unsigned long long)cap); abort(); }
  if (got && !rc) got->assign(dst.get(), dst.get() + n);
  return rc;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: codec_fuzz <corpus> [mutations]\n"); return 2; }
  const int M = argc > 2 ? atoi(argv[2]) : 300;
  std::vector<Rec> recs;
  if (!read_corpus(argv[1], recs)) { fprintf(stderr, "bad corpus\n"); return 2; }
  std::mt19937_64 rng(42);
  uint64_t ok = 0, rejected = 0, runs = 0;
  for (const Rec& r : recs) {
    std::vector<uint8_t> got;
    if (decode(r.codec, r.comp, r.orig.size(), &got) || got != r.orig) {
      fprintf(stderr, "codec %u: valid chunk of %zu bytes not decoded\n", r.codec, r.orig.size());
      return 1;
    }
    for (int m = 0; m < M; m++) {
      std::vector<uint8_t> c = r.comp;
      uint64_t cap = r.orig.size();
      switch (m % 5) {
        case 0:  // truncation
          c.resize(c.empty() ? 0 : rng() % c.size());
          break;
        case 1:  // 1-4 flipped bits
          for (int k = 0, nb = 1 + (int)(rng() % 4); k < nb && !c.empty(); k++) c[rng() % c.size()] ^= (uint8_t)(1u << (rng() % 8));
          break;
        case 2: {  // a run of random bytes
          if (c.empty()) break;
          const size_t at = rng() % c.size(), len = 1 + rng() % 16;
          for (size_t i = at; i < c.size() && i < at + len; i++) c[i] = (uint8_t)rng();
          break;
        }
        case 3:  // a smaller output buffer than the chunk decodes to
          cap = cap ? rng() % cap : 0;
          break;
        default:  // flipped bits in the first 16 bytes (headers, length prefixes, frame descriptors) + truncation
          for (int k = 0; k < 2 && !c.empty(); k++) c[rng() % std::min<size_t>(c.size(), 16)] ^= (uint8_t)(1u << (rng() % 8));
          if (c.size() > 2 && (rng() & 1)) c.resize(c.size() - 1 - rng() % (c.size() / 2));
          break;
      }
      decode(r.codec, c, cap, nullptr) ? rejected++ : ok++;
      runs++;
    }
  }
  printf("{\"records\": %zu, \"runs\": %llu, \"decoded\": %llu, \"rejected\": %llu}\n", recs.size(),
         (unsigned long long)runs, (unsigned long long)ok, (unsigned long long)rejected);
  return 0;
}
