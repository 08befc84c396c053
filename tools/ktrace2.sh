#!/bin/bash
# kernel trace summary of one bench workload: tools/ktrace2.sh <tag> <workload> [bench args]
set -o pipefail
TAG=$1; WL=$2; shift 2
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- \
  python3 $R/bench.py --workload $WL --no-cpu --steps 5 --warmup 2 "$@" > $O/${TAG}_bench.json 2> $O/${TAG}_prof.err \
  || { echo "trace failed"; tail -20 $O/${TAG}_prof.err; exit 1; }
cp $(find $O/${TAG}_prof -name '*kernel_stats.csv' | head -1) $O/${TAG}_kernel_stats.csv
python3 $R/tools/trace_summary.py $O/${TAG}_prof "pg::[a-z0-9_]+_kernel" > $O/${TAG}_trace.txt
rm -rf $O/${TAG}_prof
cat $O/${TAG}_trace.txt
