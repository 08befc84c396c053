#!/bin/bash
# config 5 (fused index count) check: the index / inverted-leaf GPU tests, then the index bench per variant library
# (tools/variant.sh pg_index builds; "base" = the main library).  Stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "index or inverted or roaring or sorted or config5 or mv or not_in or bitmap" > gpurun_out/idx_tests.log 2>&1 \
  || { echo "index tests failed"; tail -40 gpurun_out/idx_tests.log; exit 1; }
tail -2 gpurun_out/idx_tests.log
WL=index bash tools/r05_lib_sweep.sh "$@" || exit 1
for n in "$@"; do grep idx_prof gpurun_out/ls_$n.err | tail -2; done
exit 0
