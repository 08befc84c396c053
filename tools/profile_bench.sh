#!/bin/bash
# Round profile of one bench workload (run on the GPU box through gpurun):
#   1. bench.py (N=1, cpu baseline)                                  -> gpurun_out/<tag>_<wl>_bench.json
#   2. rocprofv3 --kernel-trace --stats over bench.py --no-cpu       -> gpurun_out/<tag>_<wl>_kernel_stats.csv
#   3. separate --pmc passes FETCH_SIZE / WRITE_SIZE over the scan   -> gpurun_out/<tag>_<wl>_traffic.json
# The profiled runs issue one query at a time (--inflight 1): their kernel means are the serial pass's, which bench.py's
# roofline uses.  Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r02}
WL=${2:-adanalytics}
STEPS=${3:-10}
EXTRA=${BENCH_ARGS:-}
R=$(pwd)
O=$R/gpurun_out
T=${TAG}_${WL}
# the hot-path kernels bench.py's roofline times (pre-pass + stream + scan / partition passes)
HOT="pg::(scan|stream|part_[a-z0-9]+|roaring_keys|index_count|set_lut_bits|fill_ranges|mv_scan|bitmap_not)_kernel"
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 $R/bench.py --workload $WL $EXTRA > $O/${T}_bench.json 2> $O/${T}_bench.err || { echo "bench failed"; tail -20 $O/${T}_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${T}_prof -o run -- \
  python3 $R/bench.py --workload $WL $EXTRA --no-cpu --inflight 1 --steps $STEPS --warmup 3 > $O/${T}_prof_bench.json 2> $O/${T}_prof.err \
  || { echo "kernel trace failed"; tail -20 $O/${T}_prof.err; exit 1; }
cp $(find $O/${T}_prof -name '*kernel_stats.csv' | head -1) $O/${T}_kernel_stats.csv
python3 $R/tools/trace_summary.py $O/${T}_prof "$HOT" > $O/${T}_scan_trace.txt
rm -rf $O/${T}_prof
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "$HOT" --output-format csv \
    -d $O/${T}_pmc_$C -o run -- python3 $R/bench.py --workload $WL $EXTRA --no-cpu --inflight 1 --steps 3 --warmup 1 \
    > $O/${T}_pmc_$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python3 $R/tools/pmc_summary.py "$HOT" $O/${T}_pmc_FETCH_SIZE $O/${T}_pmc_WRITE_SIZE > $O/${T}_pmc.txt
python3 $R/tools/traffic_json.py $O/${T}_pmc.txt $O/${T}_prof_bench.json > $O/${T}_traffic.json
rm -rf $O/${T}_pmc_FETCH_SIZE $O/${T}_pmc_WRITE_SIZE
echo profile-ok $T
