// pg_chunk_decompress (include/pinot_codec.h) over pg_codec.hip compiled as plain C++: the sanitized stand-in the
// CPU tests load through PINOT_CODEC_LIB (tests/test_sanitizers.py).  Test infrastructure only.
#include "../../pinot_amd/csrc/pg_codec.hip"

extern "C" int pg_chunk_decompress(uint32_t codec, const void* src, uint64_t src_len, void* dst, uint64_t dst_cap,
                                   uint64_t* out_len) {
  if ((!src && src_len) || (!dst && dst_cap) || !out_len) return PG_E_INVALID;
  const char* why = "";
  return pg::decompress_chunk(codec, (const uint8_t*)src, src_len, (uint8_t*)dst, dst_cap, out_len, &why);
}
