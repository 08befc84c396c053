#!/bin/bash
# PMC HBM traffic of the scan kernel on the config-3 (SSB) bench line: one --pmc pass per counter (GPU box only).
set -o pipefail
R=$(pwd)
O=$R/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/bench.py --no-cpu --workload ssb > $O/ssb_bench_line.json 2>/dev/null || { echo "bench failed"; exit 1; }
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "pg::scan_kernel" --output-format csv \
    -d $O/ssb_pmc_$C -o run -- python3 $R/bench.py --no-cpu --workload ssb --steps 3 --warmup 1 \
    > $O/ssb_pmc_$C.log 2>&1 || { echo "pmc $C failed"; exit 1; }
done
python3 $R/tools/pmc_summary.py "pg::scan_kernel" $O/ssb_pmc_FETCH_SIZE $O/ssb_pmc_WRITE_SIZE > $O/ssb_pmc.txt
python3 $R/tools/traffic_json.py $O/ssb_pmc.txt $O/ssb_bench_line.json > $O/ssb_traffic.json
rm -rf $O/ssb_pmc_FETCH_SIZE $O/ssb_pmc_WRITE_SIZE
echo pmc-ok
