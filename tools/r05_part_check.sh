#!/bin/bash
# partition kernels: parity tests, config-4 bench (two launches / persistent pipeline), phase profile (dev tool)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "ring_reuse or speculative_regions or radix_partitioned_group_by or config4" > gpurun_out/pc_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/pc_tests.log; exit 1; }
tail -2 gpurun_out/pc_tests.log
run() {
  local tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --workload highcard --no-cpu --no-full-parity --steps 5 --warmup 2 > gpurun_out/pc_$tag.json 2> gpurun_out/pc_$tag.err || { echo "variant $tag failed"; tail -5 gpurun_out/pc_$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/pc_$tag.json')); print('$tag', round(d['ms_per_step'],3), d['step_breakdown_ms']['scan_ms'])"
}
run unfused PG_PART_FUSED=0 && run fused_l3q128 PG_PART_LAG=3 PG_PART_QSPLITS=128 || exit 1
PINOT_GPU_LIB=$PWD/pinot_amd/libpinot_gpu_prof.so PG_PART_FUSED=0 timeout -k 10 300 python3 bench.py --workload highcard --no-cpu --no-full-parity --steps 1 --warmup 1 > gpurun_out/pc_prof.json 2> gpurun_out/pc_prof.err; grep part_prof gpurun_out/pc_prof.err | tail -3
(cd /tmp && export TMPDIR=/tmp && PG_PART_FUSED=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OLDPWD/gpurun_out/pc_kt -o run -- python3 $OLDPWD/bench.py --workload highcard --no-cpu --no-full-parity --steps 3 --warmup 1 > /dev/null 2>&1) || { echo "trace failed"; exit 1; }
python3 - <<'PY'
import csv, glob
f = glob.glob('gpurun_out/pc_kt/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'part_' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs']) / 1e6, 3), 'ms')
PY
rm -rf gpurun_out/pc_kt
