#!/bin/bash
# round 6 closing (MV keys under numGroupsLimit): smoke, the MV / raw-string tests, the GPU suite, then the closing
# profiles of all four workloads + config 2 at 16 segments (tools/r06_e.sh, TAG r06e).  First failure ends it.
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 240 --timeout-method thread --tb=short"
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 $T -m gpu tests/test_mv_group_by.py tests/test_raw_strings.py > gpurun_out/g_new.log 2>&1 || { echo "new tests failed"; tail -60 gpurun_out/g_new.log; exit 1; }
tail -1 gpurun_out/g_new.log
timeout -k 10 900 $T -m gpu tests > gpurun_out/g_gpu_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|ERROR" gpurun_out/g_gpu_tests.log | tail -5; tail -60 gpurun_out/g_gpu_tests.log; exit 1; }
tail -1 gpurun_out/g_gpu_tests.log
[ -n "$NO_PROFILE" ] && exit 0
TAG=r06e bash tools/r06_e.sh || exit 1
echo "r06_g ok"
