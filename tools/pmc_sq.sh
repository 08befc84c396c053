#!/bin/bash
# SQ counters (one pass) of the hot-path kernels of one bench workload (dev tool)
set -o pipefail
WL=${1:-highcard}; R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_LDS \
  --kernel-include-regex "${KRE:-pg::(scan|stream|part_[a-z0-9]+|index_count)_kernel}" --output-format csv -d $O/sq_$WL -o run -- \
  python3 $R/bench.py --workload $WL --no-cpu --no-full-parity --steps 2 --warmup 1 > $O/sq_$WL.log 2>&1 || { echo "pmc failed"; tail -5 $O/sq_$WL.log; exit 1; }
python3 $R/tools/pmc_summary.py "${KRE:-pg::(scan|stream|part_[a-z0-9]+|index_count)_kernel}" $O/sq_$WL > $O/sq_$WL.txt
rm -rf $O/sq_$WL
tail -14 $O/sq_$WL.txt
