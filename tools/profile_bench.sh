#!/bin/bash
# Round profile of the bench workload (run on the GPU box through gpurun):
#   1. bench.py (default: N=1, cpu baseline)                        -> gpurun_out/<tag>_bench.json
#   2. rocprofv3 --kernel-trace --stats over bench.py --no-cpu       -> gpurun_out/<tag>_kernel_stats.csv
#   3. separate --pmc passes FETCH_SIZE / WRITE_SIZE over the scan   -> gpurun_out/<tag>_traffic.json
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
TAG=${1:-r01}
STEPS=${2:-10}
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 420 python3 $R/bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_prof -o run -- \
  python3 $R/bench.py --no-cpu --steps $STEPS --warmup 3 > $O/${TAG}_prof_bench.json 2> $O/${TAG}_prof.err \
  || { echo "kernel trace failed"; exit 1; }
cp $(find $O/${TAG}_prof -name '*kernel_stats.csv' | head -1) $O/${TAG}_kernel_stats.csv
python3 $R/tools/trace_summary.py $O/${TAG}_prof "pg::scan_kernel" > $O/${TAG}_scan_trace.txt
rm -rf $O/${TAG}_prof
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "pg::scan_kernel" --output-format csv \
    -d $O/${TAG}_pmc_$C -o run -- python3 $R/bench.py --no-cpu --steps 3 --warmup 1 \
    > $O/${TAG}_pmc_$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python3 $R/tools/pmc_summary.py "pg::scan_kernel" $O/${TAG}_pmc_FETCH_SIZE $O/${TAG}_pmc_WRITE_SIZE > $O/${TAG}_pmc.txt
python3 $R/tools/traffic_json.py $O/${TAG}_pmc.txt $O/${TAG}_prof_bench.json > $O/${TAG}_traffic.json
rm -rf $O/${TAG}_pmc_FETCH_SIZE $O/${TAG}_pmc_WRITE_SIZE
echo profile-ok
