#!/bin/bash
# highcard bench per library variant (tools/variant.sh pg_part): "name:ENV=V ..." entries in $VARIANTS
set -o pipefail
mkdir -p gpurun_out
for V in $VARIANTS; do
  N=${V%%:*}; E=${V#*:}; [ "$E" = "$V" ] && E=""
  L=pinot_amd/libpinot_gpu.so; [ "$N" != "main" ] && L=pinot_amd/libpinot_gpu_$N.so
  [ -f "${L%.so}.flags" ] && echo "$N flags: $(cat ${L%.so}.flags)" | tee gpurun_out/sw_$N.flags
  env PINOT_GPU_LIB=$L ${E//,/ } timeout -k 10 300 python -u bench.py --workload highcard --steps 10 --warmup 3 --no-cpu > gpurun_out/sw_$N.json 2> gpurun_out/sw_$N.err \
    || { echo "bench $N failed"; tail -20 gpurun_out/sw_$N.err; exit 1; }
  echo "$V: $(python3 -c "import json;d=json.loads(open('gpurun_out/sw_$N.json').read().strip().splitlines()[-1]);print(round(d['ms_per_step'],3),d['step_breakdown_ms']['scan_ms'],d['step_breakdown_ms']['finalize_ms'])")"
done
for V in $TRACE; do
  N=${V%%:*}; E=${V#*:}; [ "$E" = "$V" ] && E=""
  cd /tmp && export TMPDIR=/tmp
  env PINOT_GPU_LIB=$GRAFT_REPO_ROOT/pinot_amd/libpinot_gpu_$N.so ${E//,/ } timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/tr_$N -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload highcard --no-cpu --steps 5 --warmup 2 > /dev/null 2>&1 || { echo "trace $N failed"; exit 1; }
  cd $GRAFT_REPO_ROOT
  python3 tools/trace_summary.py gpurun_out/tr_$N "pg::part_[a-z0-9_]+_kernel"; rm -rf gpurun_out/tr_$N
done
