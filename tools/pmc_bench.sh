#!/bin/bash
# PMC passes (one counter group per process) over a short bench run: tools/pmc_bench.sh <tag> <workload> <kernel-regex>
# -> gpurun_out/<tag>_pmc.txt (per-dispatch counter sums; FETCH_SIZE needs the guide's x2 for 16-B streaming reads)
set -o pipefail
TAG=$1; WL=$2; KRE=$3
R=$(pwd); O=$R/gpurun_out; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
run() {
  timeout -s KILL 240 rocprofv3 --pmc $2 --kernel-include-regex "$KRE" --output-format csv -d $O/${TAG}_$1 -o run -- \
    python3 $R/bench.py --workload $WL --no-cpu --steps 2 --warmup 1 > $O/${TAG}_$1.log 2>&1
}
run fetch "FETCH_SIZE" && run write "WRITE_SIZE" && \
run sq "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
  || { echo "pmc pass failed"; exit 1; }
python3 $R/tools/pmc_summary.py "$KRE" $O/${TAG}_fetch $O/${TAG}_write $O/${TAG}_sq > $O/${TAG}_pmc.txt
rm -rf $O/${TAG}_fetch $O/${TAG}_write $O/${TAG}_sq
cat $O/${TAG}_pmc.txt | head -40
