#!/bin/bash
# config-4 partition kernels: kernel trace + one SQ counter pass (dev tool)
set -o pipefail
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
WL=${1:-highcard}
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$WL -o run -- \
  python3 $R/bench.py --workload $WL --no-cpu --no-full-parity --steps 5 --warmup 2 > $O/kt_$WL.json 2> $O/kt_$WL.err) || { echo "trace failed"; tail -5 $O/kt_$WL.err; exit 1; }
cp $(find $O/kt_$WL -name '*kernel_stats.csv' | head -1) $O/kt_${WL}_stats.csv && rm -rf $O/kt_$WL
bash tools/pmc_sq.sh $WL
