#!/bin/bash
# kernel timeline of the last query of one bench workload (dev tool; see tools/timeline.py)
set -o pipefail
WL=${1:-highcard}; N=${2:-40}; R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace ${COPIES:+--memory-copy-trace} --output-format csv -d $O/tl_$WL -o run -- python3 $R/bench.py --workload $WL --no-cpu --steps 3 --warmup 1 $BENCH_ARGS > $O/tl_$WL.log 2>&1 || { echo "trace failed"; tail -5 $O/tl_$WL.log; exit 1; }
python3 $R/tools/timeline.py $O/tl_$WL $N > $O/tl_$WL.txt
rm -rf $O/tl_$WL
cat $O/tl_$WL.txt
