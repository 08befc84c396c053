/*
 * pinot_codec.h -- host-side chunk codecs of libpinot_gpu.so (C ABI).
 *
 * Raw (no-dictionary) forward indexes store their values in chunks compressed with the column's
 * ChunkCompressionType (pinot-segment-spi/.../compression/ChunkCompressionType.java:21-22).  The reference
 * decompresses a chunk per ChunkDecompressor (pinot-segment-local/.../io/compression/ChunkCompressorFactory.java,
 * SnappyDecompressor, LZ4Decompressor, LZ4WithLengthDecompressor, ZstandardDecompressor) each time a reader
 * touches it; here every chunk is decompressed once, when pg_column_upload makes the column resident.  This entry
 * point exposes the same decoders to the host side of the integration (segment loaders that want the values on
 * the heap), replacing ChunkDecompressor.decompress.
 *
 * Formats (third-party, not vendored in the reference; restated from their published specifications):
 *   PG_CODEC_SNAPPY            snappy-java 1.1.8.x raw block: varint length, literal / copy elements
 *   PG_CODEC_ZSTANDARD         zstd-jni 1.4.9-5: one or more Zstandard frames (RFC 8878)
 *   PG_CODEC_LZ4               lz4-java 1.8.0 LZ4 block (no frame); the decompressed size is the caller's capacity
 *   PG_CODEC_LZ4_LENGTH_PREFIXED  LZ4CompressorWithLength: 4-byte little-endian decompressed length + LZ4 block
 */
#ifndef PINOT_CODEC_H
#define PINOT_CODEC_H

#include <stddef.h>
#include <stdint.h>

#include "pinot_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef enum pg_codec {
  PG_CODEC_PASS_THROUGH = 0,
  PG_CODEC_SNAPPY = 1,
  PG_CODEC_ZSTANDARD = 2,
  PG_CODEC_LZ4 = 3,
  PG_CODEC_LZ4_LENGTH_PREFIXED = 4
} pg_codec;

/* Decompress one chunk of `src_len` bytes into `dst` (capacity `dst_cap`); *out_len receives the decompressed
 * length.  Returns PG_OK, PG_E_INVALID (corrupt input or a chunk larger than dst_cap) or PG_E_UNSUPPORTED (unknown
 * codec, zstd dictionaries).  Host memory only; needs no device. */
int pg_chunk_decompress(uint32_t codec, const void *src, uint64_t src_len, void *dst, uint64_t dst_cap,
                        uint64_t *out_len);

#ifdef __cplusplus
}
#endif
#endif /* PINOT_CODEC_H */
