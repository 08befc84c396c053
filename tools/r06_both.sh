#!/bin/bash
# config 3: the first two further stream leaves' slices loaded together (PG_STREAM_STAGE_BOTH variants) -- parity of
# the stream tests on each variant, then the serial bench A/B against the main build
set -o pipefail
mkdir -p gpurun_out
for L in both both6; do
  PINOT_GPU_LIB=$PWD/pinot_amd/libpinot_gpu_$L.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_gpu_stream.py -k "not overflow" > gpurun_out/both_t_$L.log 2>&1 || { echo "tests $L failed"; tail -30 gpurun_out/both_t_$L.log; exit 1; }
  tail -1 gpurun_out/both_t_$L.log
done
LIBS="main both both6" W=ssb BENCH_ARGS="--inflight 1" bash tools/lib_ab.sh
