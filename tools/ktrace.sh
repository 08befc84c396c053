#!/bin/bash
# per-kernel mean durations of one bench workload (dev tool)
set -o pipefail
WL=${1:-highcard}; R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/kt_$WL -o run -- python3 $R/bench.py --workload $WL --no-cpu --steps 3 --warmup 1 > $O/kt_$WL.log 2>&1 || { echo "trace failed"; tail -5 $O/kt_$WL.log; exit 1; }
python3 $R/tools/trace_summary.py $O/kt_$WL "pg::[a-z0-9_]+_kernel"
rm -rf $O/kt_$WL
