#!/bin/bash
# Average VMEM / LDS instruction latency (SQ_INST_LEVEL_* / SQ_INSTS_*, in cycles) of one bench workload's kernels
# (dev tool, one counter pass): tools/pmc_lat.sh <workload>
set -o pipefail
WL=${1:-index}; R=$(pwd); O=$R/gpurun_out; mkdir -p $O
KRE=${KRE:-pg::(scan|stream|part_[a-z0-9]+|index_count)_kernel}
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU \
  --kernel-include-regex "$KRE" --output-format csv -d $O/lat_$WL -o run -- \
  python3 $R/bench.py --workload $WL --no-cpu --no-full-parity --steps 2 --warmup 1 > $O/lat_$WL.log 2>&1 || { echo "pmc failed"; tail -5 $O/lat_$WL.log; exit 1; }
python3 $R/tools/pmc_summary.py "$KRE" $O/lat_$WL > $O/lat_$WL.txt
rm -rf $O/lat_$WL
tail -6 $O/lat_$WL.txt
