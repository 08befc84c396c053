"""AddressSanitizer / UndefinedBehaviorSanitizer runs of the host-side parsers of on-disk bytes.

* The chunk decoders of raw forward indexes (pinot_amd/csrc/pg_codec.hip: Snappy, LZ4 block / length-prefixed,
  Zstandard frames with FSE / Huffman tables) are host-only C++; tests/sanitize/Makefile builds them as plain C++ with
  -fsanitize=address,undefined.  codec_fuzz feeds every codec valid chunks and a few hundred truncated, bit-flipped,
  overwritten and short-buffer variants each, from exact-size heap blocks: any out-of-bounds access or undefined
  behaviour aborts the run.
* The same sanitized decoders (PINOT_CODEC_LIB) and a sanitized build of the C oracle (PINOT_ORACLE_LIB: its roaring /
  MV / sorted / raw-chunk / range-index readers) then run the CPU raw-index and segment-format tests in a child process
  with the sanitizer runtimes preloaded.
CPU only (no GPU); the device build of pg_codec.hip is the same source."""
import json
import os
import struct
import subprocess
import sys

import numpy as np
import pytest

from pinot_amd.segment import CHUNK_CODECS, chunk_compress

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "tests", "sanitize")
BUILD = os.path.join(SAN, "build")


@pytest.fixture(scope="module")
def sanitized():
    subprocess.run(["make", "-s", "-C", SAN], check=True)
    return BUILD


def _zstd_levels(b):
    import ctypes as C
    zs = C.CDLL("libzstd.so.1")
    zs.ZSTD_compressBound.restype = C.c_size_t
    zs.ZSTD_compress.restype = C.c_size_t
    zs.ZSTD_compress.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t, C.c_int]
    out = []
    for lvl in (-3, 1, 3, 12, 19):
        cap = zs.ZSTD_compressBound(C.c_size_t(len(b)))
        buf = C.create_string_buffer(max(cap, 1))
        n = zs.ZSTD_compress(buf, cap, b, len(b), lvl)
        out.append(buf.raw[:n])
    return out


def _payloads():
    rng = np.random.default_rng(3)
    return [b"", b"x", bytes(range(256)) * 3, np.arange(4000, dtype=">i8").tobytes(),
            (rng.integers(0, 50, 9000) * 1000).astype(">i4").tobytes(), rng.bytes(3000),
            b"The quick brown fox jumps over the lazy dog. " * 200]


def write_corpus(path):
    recs = 0
    with open(path, "wb") as f:
        for data in _payloads():
            chunks = [(CHUNK_CODECS[c], chunk_compress(CHUNK_CODECS[c], data))
                      for c in ("SNAPPY", "LZ4", "LZ4_LENGTH_PREFIXED", "ZSTANDARD")]
            if data:
                chunks += [(CHUNK_CODECS["ZSTANDARD"], z) for z in _zstd_levels(data)]
            for codec, comp in chunks:
                f.write(struct.pack("<IQQ", codec, len(data), len(comp)) + data + comp)
                recs += 1
    return recs


def _clean(stderr: str):
    assert "AddressSanitizer" not in stderr and "runtime error" not in stderr, stderr[-4000:]


def test_chunk_decoders_under_sanitizers(sanitized, tmp_path):
    corpus = tmp_path / "corpus.bin"
    recs = write_corpus(corpus)
    p = subprocess.run([os.path.join(sanitized, "codec_fuzz"), str(corpus), "300"], capture_output=True, text=True,
                       timeout=600, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1"))
    _clean(p.stderr)
    assert p.returncode == 0, p.stderr[-3000:]
    out = json.loads(p.stdout.strip().splitlines()[-1])
    assert out["records"] == recs and out["runs"] == 300 * recs
    assert out["rejected"] > 0 and out["decoded"] > 0   # both outcomes exercised


def _runtime(name):
    return subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()


def test_format_tests_with_sanitized_parsers(sanitized):
    """tests/test_raw_index.py and tests/test_formats.py (CPU part) with the sanitized codec and oracle builds."""
    env = dict(os.environ)
    env.update(LD_PRELOAD=f"{_runtime('libasan.so')} {_runtime('libubsan.so')}",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:verify_asan_link_order=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               PINOT_CODEC_LIB=os.path.join(sanitized, "libpg_codec_asan.so"),
               PINOT_ORACLE_LIB=os.path.join(sanitized, "libpinot_oracle_asan.so"))
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-m", "not gpu", "-p", "no:cacheprovider",
                        "tests/test_raw_index.py", "tests/test_formats.py", "tests/test_range_index.py",
                        "tests/test_oracle_golden.py"],
                       cwd=ROOT, capture_output=True, text=True, timeout=1200, env=env)
    _clean(p.stdout + p.stderr)
    assert p.returncode == 0, (p.stdout[-3000:], p.stderr[-3000:])
